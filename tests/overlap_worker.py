"""Rank body for tests/test_overlap_gpu.py: 2 processes share the box's one GPU over gloo and train
a fused Inception block through the bucketed, backward-overlapped PS and DDP data planes."""
import os
import traceback

import torch
import torch.distributed as dist

import gpu_ranks


def _model(kind, dev):
    from torch import nn

    from tony_amd.models import inception_v3 as iv3
    from tony_amd.models.layers import init_weights
    from tony_amd.ops.pool import global_avg_pool

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.block = {"A": lambda: iv3.InceptionA(64, 32), "C": lambda: iv3.InceptionC(64, 32)}[kind]()
            self.fc = nn.Linear(self.block.out_channels, 10)

        def forward(self, x):
            return self.fc(global_avg_pool(self.block(x)))

    return init_weights(Net(), seed=0).to(dev).to(memory_format=torch.channels_last).train()


def _data(rank, kind, dev):
    hw = {"A": 35, "C": 17}[kind]
    g = torch.Generator(device=dev).manual_seed(11 + rank)
    x = torch.randn((8, 64, hw, hw), generator=g, device=dev).to(torch.bfloat16)
    return x.contiguous(memory_format=torch.channels_last), torch.randint(0, 10, (8,), generator=g, device=dev)


def ps_run(rank, kind, overlap, bucket_mb, steps=3, graph=False):
    from tony_amd.ops import cross_entropy
    from tony_amd.parallel.ps import ParameterServer
    from tony_amd.parallel.trainer import Trainer

    dev = torch.device("cuda", torch.cuda.current_device())
    model = _model(kind, dev)
    ps = ParameterServer(model, optimizer="sgd", lr=0.05, momentum=0.9, device=dev, bucket_mb=bucket_mb,
                         bucketed_single=True)
    # graph: the step captured once and replayed natively (ops/plan.py) -- with several ranks the
    # buckets' collectives are issued between plan segments (parallel/trainer.py _replay_overlapped)
    tr = Trainer(model, ps, lambda o, y: cross_entropy(o, y), overlap_comm=overlap, use_graph=graph, warmup_eager=1)
    x, y = _data(rank, kind, dev)
    from tony_amd.parallel import collectives as coll

    fb0 = coll.fallback_count()
    for s in range(steps):
        if s == steps - 1:
            ps.engine.log = []
        tr.step(x, y)
    torch.cuda.synchronize()
    return {"params": ps.flat.data.float().cpu(), "log": ps.engine.log, "n_buckets": len(ps.buckets),
            "overlapped": ps.overlapped_buckets, "train_fallbacks": coll.fallback_count() - fb0,
            "replay": tr.replay_kind, "plan_buckets": tr.plan_buckets, "plan_error": tr.plan_error}


def ddp_run(rank, kind, bucket_mb):
    from tony_amd.ops import cross_entropy
    from tony_amd.parallel.ddp import DistributedDataParallel

    dev = torch.device("cuda", torch.cuda.current_device())
    x, y = _data(rank, kind, dev)
    # this rank's own gradient without DDP (same init, same fused kernels): the parent checks DDP's
    # averaged gradient against the mean of these over ranks -- not only that the ranks agree
    ref = _model(kind, dev)
    for p in ref.parameters():
        p.data = p.data.to(torch.bfloat16)
    cross_entropy(ref(x), y).backward()
    local = {n: p.grad.float().cpu() for n, p in ref.named_parameters()}
    del ref
    model = _model(kind, dev)
    for p in model.parameters():
        p.data = p.data.to(torch.bfloat16)
    ddp = DistributedDataParallel(model, bucket_mb=bucket_mb, device=dev)
    from tony_amd.parallel import collectives as coll

    fb0 = coll.fallback_count()  # init-time broadcasts of small / int64 buffers may fall back; buckets may not
    ddp.zero_grad()
    cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    named = {n: p.grad.float().cpu() for n, p in model.named_parameters()}
    return {"grad": ddp.flat.grad.float().cpu(), "named": named, "local": local, "n_buckets": len(ddp.reducer.buckets),
            "overlapped": ddp.reducer.overlapped_buckets, "launches": ddp.reducer.launches,
            "train_fallbacks": coll.fallback_count() - fb0}


def run(rank, world, port, q, kind, bucket_mb):
    import faulthandler

    os.makedirs("gpurun_out", exist_ok=True)
    trace = open(os.path.join("gpurun_out", f"overlap_rank{rank}.txt"), "w")
    faulthandler.enable(file=trace, all_threads=True)
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        gpu_ranks.init(rank, world)
        out = {}
        for name, fn in (("ps_overlap", lambda: ps_run(rank, kind, True, bucket_mb)),
                         ("ps_plan", lambda: ps_run(rank, kind, True, bucket_mb, graph=True)),
                         ("ps_serial", lambda: ps_run(rank, kind, False, bucket_mb)),
                         ("ddp", lambda: ddp_run(rank, kind, bucket_mb))):
            print(f"rank {rank}: {name}", file=trace, flush=True)
            out[name] = fn()
        dist.barrier()
        dist.destroy_process_group()
        # by value: a tensor would travel as a shared-memory handle that dies with this process
        from tony_amd.parallel import collectives as coll

        def val(v):
            if isinstance(v, torch.Tensor):
                return v.numpy()
            if isinstance(v, dict):
                return {k: val(x) for k, x in v.items()}
            return v

        res = {k: val(v) for k, v in out.items()}
        res["fallbacks"] = coll.fallback_count()
        q.put((rank, res))
    except Exception:  # noqa: BLE001 - reported to the parent
        q.put((rank, {"error": traceback.format_exc()}))
