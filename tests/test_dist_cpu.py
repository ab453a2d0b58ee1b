"""Multi-process data-plane tests on CPU (gloo): DDP buckets, the Horovod API, the parameter
server (colocated / dedicated sync / dedicated async), collectives and the MXNet-style kvstore.

Each test starts one process per rank (spawn), exactly as the TonY runtimes would start one
task per rank, and compares against a single-process fp32 reference.
"""
import multiprocessing as mp
import socket

import pytest
import torch

import dist_workers as W

pytestmark = pytest.mark.timeout(180)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, arglists):
    ctx = mp.get_context("spawn")
    with ctx.Pool(len(arglists)) as pool:
        res = [pool.apply_async(fn, a) for a in arglists]
        return [r.get(150) for r in res]


def _ref_grads(world):
    model = W._mlp(seed=0)
    total = None
    for r in range(world):
        model.zero_grad()
        x, y = W._batch(r)
        torch.nn.functional.cross_entropy(model(x), y).backward()
        g = [p.grad.clone() for p in model.parameters()]
        total = g if total is None else [a + b for a, b in zip(total, g)]
    return model, [t / world for t in total]


@pytest.mark.parametrize("bucket_mb", [32, 0.0005])
def test_ddp_bucketed_allreduce_matches_average(bucket_mb):
    world, port = 2, _port()
    outs = _run(W.ddp_rank, [(r, world, port, bucket_mb) for r in range(world)])
    _, ref = _ref_grads(world)
    for o in outs:
        for g, rg in zip(o["grads"], ref):
            torch.testing.assert_close(g, rg, rtol=1e-5, atol=1e-6)
    if bucket_mb < 0.001:
        assert outs[0]["n_buckets"] > 1
    assert outs[0]["launches"] == outs[0]["n_buckets"]        # the no_sync pass launched nothing
    assert not torch.allclose(outs[0]["local"][0], outs[1]["local"][0])   # no_sync grads are local
    for a, b in zip(outs[0]["params"], outs[1]["params"]):
        torch.testing.assert_close(a, b)                      # rank 0's init was broadcast


def test_hvd_api_and_distributed_optimizer():
    from tony_amd.horovod.rendezvous import RendezvousServer

    srv = RendezvousServer("127.0.0.1")
    port = srv.start()
    try:
        world = 2
        outs = _run(W.hvd_rank, [(r, world, port) for r in range(world)])
    finally:
        srv.stop()
    for r, o in enumerate(outs):
        assert (o["rank"], o["size"]) == (r, 2)
        assert o["avg"] == [1.5] * 3 and o["sum"] == [3.0] * 3 and o["max"] == [2.0] * 3
        assert o["gather"] == [0.0, 0.0, 1.0]
        assert o["bcast"] == [10.0] and o["obj"] == {"r": 0} and o["objs"] == [0, 2]
    assert outs[0]["a2a"] == [0.0, 1.0, 100.0, 101.0] and outs[1]["a2a"] == [2.0, 3.0, 102.0, 103.0]
    # two accumulated passes per rank, averaged over ranks
    model, ref = _ref_grads(2)
    for o in outs:
        for g, rg in zip(o["grads"], ref):
            torch.testing.assert_close(g, 2 * rg, rtol=1e-5, atol=1e-6)
    for a, b in zip(outs[0]["params"], outs[1]["params"]):
        torch.testing.assert_close(a, b)


def _ps_reference(workers, steps, lr=0.1, mu=0.9):
    """Sync PS semantics: grads averaged over the worker ranks, momentum SGD on fp32."""
    model = W._mlp(seed=0)
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=mu)
    for _ in range(steps):
        opt.zero_grad()
        for r in workers:
            x, y = W._batch(r)
            (torch.nn.functional.cross_entropy(model(x), y) / len(workers)).backward()
        opt.step()
    return model


@pytest.mark.parametrize("mode,world,workers,bucket_mb,ps_ranks,overlap", [
    ("colocated", 2, [0, 1], 32, (0,), False),
    ("colocated", 3, [0, 1, 2], 0.0003, (0,), True),       # several buckets, 3-way split, launched in backward
    ("dedicated", 3, [1, 2], 32, (0,), False),
    ("dedicated", 4, [2, 3], 0.0003, (0, 1), True),        # 2 ps tasks own alternate buckets
    ("colocated", 8, list(range(8)), 0.0003, (0,), True),  # the driver's 8-GPU layout: 8 shards per bucket
])
def test_parameter_server_sync(mode, world, workers, bucket_mb, ps_ranks, overlap):
    port, steps = _port(), 3
    outs = _run(W.ps_rank, [(r, world, port, mode, True, steps, bucket_mb, ps_ranks, overlap)
                            for r in range(world)])
    ref = _ps_reference(workers, steps)
    for o in outs:
        got = o["data"]
        # compare parameter values at each slot (flat buffer is padded per tensor)
        for (off, n), p in zip(o["slots"], ref.parameters()):
            torch.testing.assert_close(got[off:off + n], p.detach().reshape(-1), rtol=1e-4, atol=1e-5)
    if bucket_mb < 0.001:
        assert outs[0]["n_buckets"] > 1
    if overlap:
        for o, r in zip(outs, range(world)):
            if r in workers:
                # every bucket but the last (the first layer's) went out while backward was still running
                assert all(k >= o["n_buckets"] - 1 for k in o["overlapped"]), o["overlapped"]
                launches = [e for e in o["log"] if e.startswith("launch:")]
                assert launches[:o["n_buckets"]] == [f"launch:{i}" for i in range(o["n_buckets"])]
                first_launch = o["log"].index("launch:0")
                assert any(e.startswith("ready:") for e in o["log"][first_launch:o["log"].index("launch:1")]) \
                    if o["n_buckets"] > 1 else True


def test_bucket_engine_order_and_double_report():
    from tony_amd.parallel.buckets import GradBucketEngine, make_buckets
    from tony_amd.parallel.flat import FlatParams

    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 8), torch.nn.Linear(8, 8))
    flat = FlatParams(model, dtype=torch.float32)
    buckets = make_buckets(flat, bucket_mb=64 * 4 / 2 ** 20 * 1.5)   # ~1.5 padded params per bucket
    assert [b.index for b in buckets] == list(range(len(buckets))) and len(buckets) >= 3
    assert buckets[0].hi == flat.numel and buckets[-1].lo == 0
    covered = sorted(i for b in buckets for i in b.params)
    assert covered == list(range(len(flat.slots)))
    seen = []
    eng = GradBucketEngine(flat, buckets, lambda b: seen.append(b.index))
    eng.begin(overlap=True)
    params = flat.params
    # report the FIRST layer's parameters first: nothing may launch before bucket 0 is complete
    eng.ready(params[:2])
    assert seen == []
    eng.ready(params[2:])
    assert seen == list(range(len(buckets)))
    with pytest.raises(RuntimeError, match="written again"):
        eng.ready(params[-1:])
    eng.end()
    assert eng.launches == len(buckets)


def test_parameter_server_async_applies_every_push():
    world, port, steps = 3, _port(), 2
    outs = _run(W.ps_rank, [(r, world, port, "dedicated", False, steps) for r in range(world)])
    ps = [o for o in outs if o["is_ps"]][0]
    init = torch.cat([p.detach().reshape(-1) for p in W._mlp(seed=0).parameters()])
    assert not torch.allclose(ps["data"][:init.numel()], init)   # updates were applied
    assert torch.isfinite(ps["data"]).all()


def test_collectives_gloo():
    world, port = 2, _port()
    outs = _run(W.collectives_rank, [(r, world, port) for r in range(world)])
    base = torch.arange(8, dtype=torch.float32)
    for r, o in enumerate(outs):
        exp = (2 * base + 1)[r * 4:(r + 1) * 4]
        assert o["rs"] == exp.tolist()
        assert o["ag"] == [0.0] * 4 + [1.0] * 4
        assert o["max"] == 1.0


@pytest.mark.parametrize("kind", ["dist_sync", "dist_async"])
def test_kvstore_dist_scheduler_server_workers(kind):
    port, steps = _port(), 3
    args = [("scheduler", 0, 1, 2, port, kind, steps), ("server", 0, 1, 2, port, kind, steps),
            ("worker", 0, 1, 2, port, kind, steps), ("worker", 1, 1, 2, port, kind, steps)]
    outs = _run(W.kv_rank, args)
    workers = [o for o in outs if o["role"] == "worker"]
    assert sorted(o["rank"] for o in workers) == [0, 1] and workers[0]["n"] == 2
    for o in workers:
        assert o["k7"] == [1.0, 1.0]
    if kind == "dist_sync":
        # every round: grad = sum of pushes (1+2) * rescale 1/2 = 1.5 ; w -= 0.5*1.5
        for o in workers:
            for s, w in enumerate(o["seen"]):
                torch.testing.assert_close(w, torch.full((3,), -0.75 * (s + 1)))
    else:
        # async: every push applied on arrival, w -= 0.5 * 0.5 * v; 3 pushes of 1 and 3 of 2 -> -2.25 after
        # the globally last push, which the worker that made it sees on its last pull
        final = min(float(o["seen"][-1][0]) for o in workers)
        assert final == pytest.approx(-2.25)


def test_kvstore_local_and_optimizer_state(tmp_path):
    import tony_amd.kv as kv

    s = kv.create("local")
    s.init(3, torch.zeros(2))
    s.push(3, [torch.ones(2), torch.ones(2)])       # multi-device push is summed
    out = torch.empty(2)
    s.pull(3, out=out)
    assert out.tolist() == [2.0, 2.0]
    s.set_optimizer(kv.create_optimizer("sgd", learning_rate=0.1, momentum=0.9))
    s.push(3, torch.ones(2))
    s.pull(3, out=out)
    torch.testing.assert_close(out, torch.tensor([1.9, 1.9]))
    s.save_optimizer_states(str(tmp_path / "opt.pt"))
    s2 = kv.create("local")
    s2.load_optimizer_states(str(tmp_path / "opt.pt"))
    assert "mom" in s2._opt.state[3]


def test_bucket_engine_inplace_report_then_accumulate_hook():
    """A fused op accumulates in place, reports, returns None -- and AccumulateGrad's hook still fires
    right after: the repeat is ignored, buckets launch in order during backward."""
    from tony_amd.ops import _lib
    from tony_amd.parallel.buckets import GradBucketEngine, make_buckets
    from tony_amd.parallel.flat import FlatParams

    class InPlaceMul(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            ctx.params = (w,)
            ctx.save_for_backward(x)
            return x * w

        @staticmethod
        def backward(ctx, g):
            (x,) = ctx.saved_tensors
            w = ctx.params[0]
            w.grad.add_((g * x).sum(0))
            _lib.report_inplace(ctx.params, (None,))
            return g * w, None

    m = torch.nn.Module()
    m.w1 = torch.nn.Parameter(torch.ones(64))
    m.w2 = torch.nn.Parameter(torch.ones(64))
    flat = FlatParams(m, dtype=torch.float32)
    seen = []
    eng = GradBucketEngine(flat, make_buckets(flat, 64 * 4 / 2 ** 20), lambda b: seen.append(b.index))
    eng.attach()
    eng.log = []
    eng.begin(overlap=True)
    x = torch.ones(2, 64, requires_grad=True)
    InPlaceMul.apply(InPlaceMul.apply(x, m.w1), m.w2).sum().backward()
    eng.end()
    assert seen == [0, 1]
    assert eng.log == ["ready:w2", "launch:0", "ready:w1", "launch:1"]
    assert eng.launched_during_backward == 2
    torch.testing.assert_close(m.w1.grad, torch.full((64,), 2.0))
    eng.detach()


def test_kvstore_plane_layout_agrees_between_server_and_workers(monkeypatch):
    """The GPU payload plane's window layout (parallel/kvstore.py _KvLayout): a server that sees only its
    own keys places them exactly where every worker (which sees all keys) expects them; a key too big for
    the window stays on gloo for everybody; rows and landing slots are 16-B aligned and disjoint."""
    from tony_amd.parallel.kvstore import _KvLayout, _Topology

    monkeypatch.setenv("DMLC_NUM_SERVER", "2")
    monkeypatch.setenv("DMLC_NUM_WORKER", "3")
    topo = _Topology()
    window = 4096
    keys = [(0, 12), (1, 100), (2, 200), (3, 8), (4, 5000), (5, 40)]  # key 4 fits no window
    worker = _KvLayout(topo, window)
    fits = {k: worker.add_key(k, n) for k, n in keys}
    assert fits == {0: True, 1: True, 2: True, 3: True, 4: False, 5: True}
    for s in range(2):
        server = _KvLayout(topo, window)
        for k, n in keys:
            if topo.server_of(k) == s:
                assert server.add_key(k, n) == fits[k]
                if fits[k]:
                    assert server.keys[k] == worker.keys[k]
    spans, slots = {}, {}
    for k, (s, n, row, land, slot) in worker.keys.items():
        assert row % 16 == 0 and land % 16 == 0 and land // worker.region == s
        slots.setdefault(s, []).append(slot)  # each server's device-flag slots: 0, 1, ... in init order
        spans.setdefault(("row", s), []).append((row, row + 3 * ((n + 15) // 16 * 16)))
        spans.setdefault(("land",), []).append((land, land + n))
    for v in spans.values():
        v.sort()
        assert all(a[1] <= b[0] for a, b in zip(v, v[1:]))
    assert all(v == list(range(len(v))) for v in slots.values())


def test_kv_server_parks_a_plane_push_that_arrives_before_init(monkeypatch):
    """A worker's plane push (OP_PUSH_X) can reach the server before worker 0's INIT of the key: the
    server has no window row for the key yet, so it must park the raw header and read the row when
    the INIT has laid the key out -- not raise KeyError.  A stand-in plane over host memory."""
    import ctypes

    from tony_amd.parallel import kvstore as kvs

    monkeypatch.setenv("DMLC_ROLE", "server")
    monkeypatch.setenv("DMLC_NUM_SERVER", "1")
    monkeypatch.setenv("DMLC_NUM_WORKER", "2")
    topo = kvs._Topology()
    window = torch.zeros(4096, dtype=torch.uint8)

    class HostPlane:
        device = torch.device("cpu")
        base = window.data_ptr()

        def __init__(self):
            self.layout = kvs._KvLayout(topo, window.numel())
            self.keys = self.layout.keys
            self.copies = []

        def add_key(self, kid, nbytes):
            return self.layout.add_key(kid, nbytes)

        def take(self, kid, w, numel, dtype):  # _KvPlane.take without the device flag wait
            _, nbytes, row_off, _, _ = self.keys[kid]
            buf = torch.empty(numel, dtype=dtype)
            self.copies.append(nbytes)
            ctypes.memmove(buf.data_ptr(), self.base + row_off + w * kvs._pad16(nbytes), nbytes)
            return buf, None

    plane = HostPlane()
    srv = kvs._Server(topo, sync=False, plane=plane)
    kid, n = 5, 3
    # worker 1 (global rank 2) wrote its row -- at the offset the layout WILL give the key -- then sent the header
    lay = kvs._KvLayout(topo, window.numel())
    lay.add_key(kid, 4 * n)
    _, nbytes, row_off, _, _ = lay.keys[kid]
    row = torch.tensor([1.0, 2.0, 3.0])
    ctypes.memmove(window.data_ptr() + row_off + 1 * kvs._pad16(nbytes), row.data_ptr(), nbytes)
    assert srv.handle(2, [kvs.OP_PUSH_X, kid, n, kvs._dcode(torch.float32)]) is True
    assert kid in srv.early and plane.copies == []           # parked, the row not read yet
    srv.handle(1, [kvs.OP_INIT, kid, n, kvs._dcode(torch.float32)], torch.zeros(n))
    assert kid not in srv.early
    # async server without an optimizer: the pushed value replaces the stored one
    torch.testing.assert_close(srv.values[kid].cpu(), row)
    assert plane.copies == [nbytes]
