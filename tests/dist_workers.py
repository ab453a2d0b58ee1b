"""Rank bodies for the multi-process (gloo, CPU) data-plane tests.  Each returns a picklable result."""
import os

import torch
import torch.distributed as dist


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TONY_DIST_BACKEND="gloo")
    from tony_amd.parallel.bootstrap import init_from_env

    return init_from_env()


def _mlp(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))


def _batch(rank, n=6):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(n, 8, generator=g), torch.randint(0, 4, (n,), generator=g)


def ddp_rank(rank, world, port, bucket_mb):
    from tony_amd.parallel.ddp import DistributedDataParallel

    _init(rank, world, port)
    model = DistributedDataParallel(_mlp(seed=rank), bucket_mb=bucket_mb)  # different init: rank 0 wins
    x, y = _batch(rank)
    loss = torch.nn.functional.cross_entropy(model(x), y)
    loss.backward()
    grads = [p.grad.clone() for p in model.module.parameters()]
    # accumulation: two passes under no_sync + one synced pass
    model.zero_grad()
    with model.no_sync():
        torch.nn.functional.cross_entropy(model(x), y).backward()
    local_only = [p.grad.clone() for p in model.module.parameters()]
    out = dict(grads=grads, local=local_only, params=[p.detach().clone() for p in model.module.parameters()],
               launches=model.reducer.launches, n_buckets=len(model.reducer.buckets))
    dist.destroy_process_group()
    return out


def hvd_rank(rank, world, rdv_port):
    os.environ.update(HOROVOD_RANK=str(rank), HOROVOD_SIZE=str(world), HOROVOD_LOCAL_RANK=str(rank),
                      HOROVOD_LOCAL_SIZE=str(world), HOROVOD_GLOO_RENDEZVOUS_ADDR="127.0.0.1",
                      HOROVOD_GLOO_RENDEZVOUS_PORT=str(rdv_port), TONY_DIST_BACKEND="gloo")
    import tony_amd.hvd as hvd

    hvd.init()
    out = {"rank": hvd.rank(), "size": hvd.size()}
    t = torch.full((3,), float(rank + 1))
    out["avg"] = hvd.allreduce(t).tolist()
    out["sum"] = hvd.allreduce(t, op=hvd.Sum).tolist()
    out["max"] = hvd.allreduce(t, op=hvd.Max).tolist()
    out["gather"] = hvd.allgather(torch.arange(rank + 1, dtype=torch.float32)).tolist()
    out["bcast"] = hvd.broadcast(torch.tensor([rank * 10.0]), root_rank=1).tolist()
    out["obj"] = hvd.broadcast_object({"r": rank}, root_rank=0)
    out["objs"] = hvd.allgather_object(rank * 2)
    out["a2a"] = hvd.alltoall(torch.arange(world * 2, dtype=torch.float32) + 100 * rank).tolist()
    model = _mlp(seed=rank)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), backward_passes_per_step=2)
    for _ in range(2):
        x, y = _batch(rank)
        torch.nn.functional.cross_entropy(model(x), y).backward()
    out["grads"] = [p.grad.clone() for p in model.parameters()]
    opt.step()
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    out["params"] = [p.detach().clone() for p in model.parameters()]
    hvd.shutdown()
    return out


def ps_rank(rank, world, port, mode, sync, steps, bucket_mb=32, ps_ranks=(0,), overlap=False, wire=None):
    from tony_amd.parallel.ps import ParameterServer

    _init(rank, world, port)
    model = _mlp(seed=rank)
    ps = ParameterServer(model, optimizer="sgd", lr=0.1, momentum=0.9, mode=mode, sync=sync, dtype=torch.float32,
                         ps_ranks=ps_ranks, bucket_mb=bucket_mb, wire_dtype=wire)
    ps.engine.log = []
    overlapped = []
    if mode == "dedicated" and not sync and ps.is_ps:
        ps.serve_async(total_pushes=steps * (world - 1))
    else:
        for _ in range(steps):
            if ps.is_worker:
                ps.zero_grad()
                if overlap:
                    ps.begin_step(overlap=True)  # buckets launch from the AccumulateGrad hooks
                x, y = _batch(rank)
                torch.nn.functional.cross_entropy(model(x), y).backward()
                overlapped.append(ps.overlapped_buckets)
            ps.step()
    dist.barrier()
    out = {"data": ps.flat.data.clone(), "is_ps": ps.is_ps, "n_buckets": len(ps.buckets), "log": ps.engine.log,
           "overlapped": overlapped, "slots": [(s.offset, s.numel) for s in ps.flat.slots],
           "sd": ps.state_dict()}
    dist.destroy_process_group()
    return out


def collectives_rank(rank, world, port):
    from tony_amd.parallel import collectives as coll

    _init(rank, world, port)
    inp = torch.arange(world * 4, dtype=torch.float32) + rank
    out = torch.empty(4)
    coll.reduce_scatter_flat(out, inp.clone())
    gathered = torch.empty(world * 4)
    coll.all_gather_flat(gathered, torch.full((4,), float(rank)))
    mx = coll.max_over_ranks(float(rank))
    dist.destroy_process_group()
    return {"rs": out.tolist(), "ag": gathered.tolist(), "max": mx}


def kv_rank(role, index, num_servers, num_workers, port, kind, steps, device="cpu"):
    os.environ.update(DMLC_ROLE=role, DMLC_NUM_SERVER=str(num_servers), DMLC_NUM_WORKER=str(num_workers),
                      DMLC_PS_ROOT_URI="127.0.0.1", DMLC_PS_ROOT_PORT=str(port), TASK_INDEX=str(index))
    if device == "cpu":
        os.environ["TONY_KV_PLANE"] = "gloo"
    import tony_amd.kv as kv

    if kv.run_role():
        return {"role": role}
    store = kv.create(kind)
    w = torch.zeros(3, device=device)
    store.init("w", w)
    store.init(7, torch.ones(2, device=device))
    big_n = 1000003  # not a multiple of 16 bytes: the copy kernel's tail
    store.init("big", torch.zeros(big_n, device=device))
    store.set_optimizer(kv.create_optimizer("sgd", learning_rate=0.5, rescale_grad=1.0 / num_workers))
    seen = []
    big = torch.empty(big_n, device=device)
    ramp = torch.arange(big_n, dtype=torch.float32, device=device) / big_n
    for s in range(steps):
        store.push("w", torch.full((3,), float(store.rank + 1), device=device))
        store.push("big", ramp * (store.rank + 1))
        store.pull("w", out=w)
        store.pull("big", out=big)
        seen.append(w.clone().cpu())
    out2 = torch.empty(2, device=device)
    store.pull(7, out=out2)
    res = {"role": role, "rank": store.rank, "seen": seen, "k7": out2.tolist(), "n": store.num_workers,
           "big": big.cpu(), "plane_ops": list(getattr(store, "plane_ops", [0, 0]))}
    store.close()
    return res


def kv_bulk_rank(role, index, num_servers, num_workers, port, kind, steps, keys, key_mb):
    """``keys`` keys of ``key_mb`` MB each through the kvstore GPU plane; per-step wall time of one
    push-all + pull-all round (the host never waits for a payload: timed to a device synchronize)."""
    import time

    os.environ.update(DMLC_ROLE=role, DMLC_NUM_SERVER=str(num_servers), DMLC_NUM_WORKER=str(num_workers),
                      DMLC_PS_ROOT_URI="127.0.0.1", DMLC_PS_ROOT_PORT=str(port), TASK_INDEX=str(index),
                      TONY_KV_WINDOW_MB=str(num_workers * keys * key_mb + 64))
    import tony_amd.kv as kv

    if kv.run_role():
        return {"role": role}
    store = kv.create(kind)
    n = key_mb * (1 << 20) // 4
    vals = [torch.zeros(n, device="cuda") for _ in range(keys)]
    for k, v in enumerate(vals):
        store.init(k, v)
    store.set_optimizer(kv.create_optimizer("sgd", learning_rate=0.5, rescale_grad=1.0 / num_workers))
    ramp = torch.arange(n, dtype=torch.float32, device="cuda") / n
    grads = [ramp * (store.rank + 1) + k for k in range(keys)]
    times = []
    for _ in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(keys):
            store.push(k, grads[k])
        for k in range(keys):
            store.pull(k, out=vals[k])
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    res = {"role": role, "rank": store.rank, "times": times, "plane_ops": list(store.plane_ops),
           "v0": vals[0][:: n // 64].cpu(), "vlast": vals[-1][:: n // 64].cpu(), "n": n}
    store.close()
    return res


def kv_pullpull_rank(role, index, num_servers, num_workers, port, rounds):
    """dist_async on the GPU plane: worker 0 only pulls, twice in a row per round (no push of its own in
    between -- the pull-pull case of ADVICE r5), while worker 1 keeps pushing.  Every pulled tensor must be
    one consistent version -w_k = -0.25 k ramp (lr 0.5 x rescale 1/2 per push): a copy-out that overlapped
    the server's next reply would mix two k across the tensor."""
    os.environ.update(DMLC_ROLE=role, DMLC_NUM_SERVER=str(num_servers), DMLC_NUM_WORKER=str(num_workers),
                      DMLC_PS_ROOT_URI="127.0.0.1", DMLC_PS_ROOT_PORT=str(port), TASK_INDEX=str(index))
    import tony_amd.kv as kv

    if kv.run_role():
        return {"role": role}
    store = kv.create("dist_async")
    n = 1 << 20  # 4 MiB: 1024 flag adds per copy
    store.init("big", torch.zeros(n, device="cuda"))
    store.set_optimizer(kv.create_optimizer("sgd", learning_rate=0.5, rescale_grad=1.0 / num_workers))
    ramp = (torch.arange(n, dtype=torch.float32, device="cuda") + 1) / n
    torn, ks = 0, []
    if store.rank == 1:
        for _ in range(rounds):
            store.push("big", ramp)
    else:
        outs = [torch.empty(n, device="cuda") for _ in range(2)]
        for _ in range(rounds):
            store.pull("big", out=outs[0])
            store.pull("big", out=outs[1])
            for o in outs:
                k = torch.round(-o / (0.25 * ramp))
                ks.append(int(k[0].item()))
                torn += int((k != k[0]).any().item())
    res = {"role": role, "rank": store.rank, "torn": torn, "ks": ks,
           "plane_ops": list(getattr(store, "plane_ops", [0, 0]))}
    store.close()
    return res
