"""One-command JSON benchmarks of the BASELINE.json configs other than the Inception-v3 PS headline.

``python bench.py --config NAME [--gpus N --steps K --warmup W]`` -- the same contract as the headline
(bench.py): N ranks on one node (one per GPU), W untimed warmup steps, K timed steps bracketed by a barrier
plus a device synchronisation on both sides, the MAX over ranks, ONE JSON line from rank 0, the exit code of
the run.  A collective that falls back from the requested data plane fails the run loudly.

``hvd-resnet50``   horovod-on-tony ResNet-50 ring-allreduce bf16 (BASELINE: 8x MI355X): the fused-kernel
                   ResNet-50 through the Horovod API (``tony_amd.hvd``: ``DistributedOptimizer``'s bucketed
                   all-reduce on RCCL, overlapped with backward), per-rank batch 128 at 224x224, SGD-momentum.
                   Reference contract: ``tony-core/.../runtime/HorovodRuntime.java:318-349`` (HOROVOD_* env)
                   and ``tony-examples/horovod-on-tony/tensorflow2_mnist.py:73`` (DistributedGradientTape).
``ddp-mnist``      tony-examples/mnist-pytorch DistributedDataParallel, 8 workers (BASELINE): the reference's
                   ``Linear(784, 10)`` (``mnist_distributed.py:129-136``), batch 128 per rank (``:220``), SGD
                   lr 0.01 momentum 0.5, gradients averaged by tony_amd's bucketed DDP (one flat all-reduce per
                   step instead of the reference's per-parameter CPU all_reduce, ``:113-126``).
``mxnet-kv``       tony-examples/linearregression-mxnet with ``kvstore=dist_sync``, 1 server + N workers
                   (BASELINE: 8 workers): FullyConnected(num_hidden=1) on scalar rows, batch 1024 per worker
                   (``mxnet_dist_ex.py:35-37,50,61-68``); every step pushes the weight / bias gradients to the
                   server, which sums the round and applies SGD, and pulls the new values.  A scheduler, the
                   server and the workers run as separate processes with the DMLC_* env of TonY's mxnet runtime
                   (``MXNetRuntime.java:44-66``).

Data is synthetic and weights are random-init (no network for datasets).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time

CONFIGS = ("hvd-resnet50", "ddp-mnist", "mxnet-kv")


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _timed(step, steps: int, warmup: int, dev, world: int) -> float:
    """Seconds for ``steps`` calls of ``step`` after ``warmup`` untimed ones: barrier + synchronize on both
    sides, the max over ranks (the whole job runs at its slowest rank's pace)."""
    import torch
    import torch.distributed as dist

    from .parallel.collectives import max_over_ranks

    cuda = dev.type == "cuda"
    for _ in range(warmup):
        step()
    if cuda:
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    if cuda:
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if cuda:
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    return max_over_ranks(time.perf_counter() - t0, device=dev)


def _record(metric, value, unit, world, args, ms, dtype, data, config) -> dict:
    return {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": dtype, "data": data, "config": config}


def _init_ranks():
    """The rank's process group (env:// from torch.distributed.run, or a single rank) and its GPU."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        dev = torch.device("cuda", int(os.environ.get("TONY_BENCH_DEVICE", local % torch.cuda.device_count())))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    backend = os.environ.get("TONY_BENCH_BACKEND", "nccl" if dev.type == "cuda" else "gloo")
    if not dist.is_initialized():
        kw = {"device_id": dev} if backend == "nccl" else {}
        if world > 1:
            dist.init_process_group(backend, **kw)
        else:  # one rank: a private store, no rendezvous port
            dist.init_process_group(backend, store=dist.HashStore(), rank=0, world_size=1, **kw)
    return rank, world, dev


def hvd_resnet50(args) -> int:
    import torch

    import tony_amd.hvd as hvd
    from .jobs.common import synthetic_images
    from .models.layers import cast_model
    from .models.resnet import resnet50
    from .ops import cross_entropy
    from .parallel import collectives as coll

    rank, world, dev = _init_ranks()
    hvd.init()  # on the process group above (HOROVOD_* env when TonY launches it: jobs/hvd_resnet50.py)
    on_gpu = dev.type == "cuda"
    dtype = torch.bfloat16 if on_gpu else torch.float32
    model = cast_model(resnet50(fused=on_gpu, seed=0), dtype, dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.1 * world, momentum=0.9, weight_decay=5e-5)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), bucket_mb=args.bucket_mb or 32)
    x, y = synthetic_images(args.batch, 224, 1000, dev, dtype, seed=rank)
    xent = cross_entropy if on_gpu else (lambda o, t: torch.nn.functional.cross_entropy(o.float(), t))
    loss = [None]

    def step():
        opt.zero_grad()
        loss[0] = xent(model(x), y)
        loss[0].backward()
        opt.step()

    hvd.broadcast_parameters(model.state_dict(), root_rank=0)  # the reference jobs' first-step sync (K6)
    el = _timed(step, args.steps, args.warmup, dev, world)
    fin = float(loss[0].float().item())
    if rank == 0:
        print(json.dumps(_record(
            "images/sec (whole node) ResNet-50 Horovod ring-allreduce", args.batch * world * args.steps / el,
            "images/sec", world, args, 1000 * el / args.steps, "bf16" if on_gpu else "fp32",
            "synthetic ImageNet-shaped 224x224x3 batches, random-init weights",
            {"model": "resnet50", "global_batch": args.batch * world, "per_gpu_batch": args.batch, "seq_len": None,
             "parallelism": f"dp{world} (hvd.DistributedOptimizer: bucketed all-reduce overlapped with backward)",
             "collective": "hip-xgmi" if coll.use_hip() else "rccl", "collective_fallbacks": coll.fallback_count(),
             "optimizer": "SGD-momentum (fused HIP apply per flat buffer)", "final_loss": round(fin, 4),
             "kernels": "tony_amd HIP" if on_gpu else "cpu"})), flush=True)
    return _fallback_rc(coll) or (0 if fin == fin else 3)


def ddp_mnist(args) -> int:
    import torch

    from .models.mnist import mnist_model, synthetic_mnist
    from .parallel import collectives as coll
    from .parallel.ddp import DistributedDataParallel

    rank, world, dev = _init_ranks()
    model = mnist_model("linear", seed=0).to(dev)
    ddp = DistributedDataParallel(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.5)
    x_all, y_all = synthetic_mnist(args.batch * world, seed=1, device=dev)
    x, y = x_all[rank * args.batch:(rank + 1) * args.batch], y_all[rank * args.batch:(rank + 1) * args.batch]
    loss = [None]

    def step():
        ddp.zero_grad()
        loss[0] = torch.nn.functional.cross_entropy(ddp(x), y)
        loss[0].backward()
        opt.step()

    el = _timed(step, args.steps, args.warmup, dev, world)
    fin = float(loss[0].item())
    if rank == 0:
        print(json.dumps(_record(
            "samples/sec (whole node) MNIST PyTorch DDP", args.batch * world * args.steps / el, "samples/sec",
            world, args, 1000 * el / args.steps, "fp32", "synthetic MNIST-shaped 28x28 batches (fixed teacher labels)",
            {"model": "mnist linear 784->10 (mnist_distributed.py)", "global_batch": args.batch * world,
             "per_gpu_batch": args.batch, "seq_len": None,
             "parallelism": f"dp{world} (bucketed DDP: one flat gradient all-reduce per step)",
             "collective": "hip-xgmi" if coll.use_hip() else ("rccl" if dev.type == "cuda" else "gloo"),
             "collective_fallbacks": coll.fallback_count(), "final_loss": round(fin, 4)})), flush=True)
    return _fallback_rc(coll) or (0 if fin == fin else 3)


def _fallback_rc(coll) -> int:
    if coll.use_hip() and coll.fallback_count():
        print(f"bench: TONY_COLLECTIVE=hip requested but {coll.fallback_count()} collectives fell back to RCCL",
              file=sys.stderr, flush=True)
        return 4
    return 0


def mxnet_kv_worker(args) -> int:
    """One worker of the mxnet-kv bench (DMLC_ROLE=worker; the scheduler / server roles serve and exit)."""
    import torch
    import torch.distributed as dist

    import tony_amd.kv as kv

    if kv.run_role():
        return 0
    store = kv.create(args.kvstore)
    rank, nw = store.rank, store.num_workers
    use_gpu = args.kv_device == "cuda" or (args.kv_device == "auto" and torch.cuda.is_available())
    dev = torch.device("cuda", torch.cuda.current_device()) if use_gpu else torch.device("cpu")
    g = torch.Generator().manual_seed(rank)
    xb = (torch.rand(args.batch, 1, generator=g) * 2 - 1).to(dev)
    yb = 3.0 * xb[:, 0] + 0.5
    w, b = torch.zeros(1, 1, device=dev), torch.zeros(1, device=dev)
    store.init("fc_weight", w)
    store.init("fc_bias", b)
    store.set_optimizer(kv.create_optimizer("sgd", learning_rate=0.1, rescale_grad=1.0 / (args.batch * nw)))

    def step():
        err = (xb @ w.t())[:, 0] + b - yb
        store.push("fc_weight", 2 * (err[:, None] * xb).sum(0, keepdim=True))
        store.push("fc_bias", 2 * err.sum(0, keepdim=True))
        store.pull("fc_weight", out=w)
        store.pull("fc_bias", out=b)

    for _ in range(args.warmup):
        step()
    if use_gpu:
        torch.cuda.synchronize(dev)
    store.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if use_gpu:
        torch.cuda.synchronize(dev)
    store.barrier()
    el = torch.tensor([time.perf_counter() - t0])
    dist.all_reduce(el, op=dist.ReduceOp.MAX, group=store.workers)
    el = float(el)
    mse = float(((xb @ w.t())[:, 0] + b - yb).pow(2).mean())
    ops = list(getattr(store, "plane_ops", [0, 0]))
    store.close()
    if rank == 0:
        print(json.dumps(_record(
            "samples/sec (whole node) MXNet linear regression kvstore", args.batch * nw * args.steps / el,
            "samples/sec", nw, args, 1000 * el / args.steps, "fp32",
            "synthetic rows y = 3x + 0.5, random-init (zero) weights",
            {"model": "FullyConnected(num_hidden=1) (mxnet_dist_ex.py)", "global_batch": args.batch * nw,
             "per_gpu_batch": args.batch, "seq_len": None, "kvstore": args.kvstore,
             "parallelism": f"1 server + {nw} workers ({args.kvstore}), scheduler process",
             "tensors_on": dev.type, "plane_pushes_pulls_rank0": ops, "final_mse": round(mse, 6)})), flush=True)
    return 0 if mse == mse else 3  # (a short bench run need not converge; a NaN is a failure)


def mxnet_kv_launch(args, argv) -> int:
    """Scheduler + 1 server + N workers as child processes with TonY's mxnet env contract; relays worker
    0's JSON line (inherited stdout) and returns the worst exit code."""
    port = _free_port()
    n = args.gpus
    base = dict(os.environ, DMLC_PS_ROOT_URI="127.0.0.1", DMLC_PS_ROOT_PORT=str(port), DMLC_NUM_SERVER="1",
                DMLC_NUM_WORKER=str(n), HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        base.pop(k, None)
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    child_argv = [a for a in argv if a != "--launch-dry-run"] + ["--kv-role-child"]
    roles = [("scheduler", 0), ("server", 0)] + [("worker", i) for i in range(n)]
    plan = []
    for role, idx in roles:
        env = dict(base, DMLC_ROLE=role, TASK_INDEX=str(idx), JOB_NAME=role)
        if role != "worker":
            env["TONY_KV_DEVICE"] = os.environ.get("TONY_BENCH_DEVICE", "0")  # the server shares a GPU
        else:  # worker i on GPU i (every GPU visible: the payload plane maps peer windows)
            env["TONY_KV_WORKER_DEVICE"] = os.environ.get("TONY_BENCH_DEVICE", str(idx))
        plan.append((role, idx, env))
    if args.launch_dry_run:
        print(json.dumps({"mxnet_kv_launch": [[r, i, {k: e[k] for k in ("DMLC_ROLE", "TASK_INDEX", "DMLC_NUM_WORKER",
                                                                         "DMLC_NUM_SERVER")}] for r, i, e in plan]}))
        return 0
    procs = [subprocess.Popen([sys.executable, script] + child_argv, env=e,
                              stdout=None if r == "worker" else subprocess.DEVNULL) for r, _, e in plan]
    rc = 0
    deadline = time.time() + float(os.environ.get("TONY_BENCH_KV_TIMEOUT_S", "900"))
    for p in procs:
        try:
            c = p.wait(timeout=max(1.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            return 124
        rc = rc or c
    return rc


def run(args, argv) -> int:
    """bench.py's --config dispatch (after its own self-launch of N ranks for the torchrun configs)."""
    if args.config == "hvd-resnet50":
        return hvd_resnet50(args)
    if args.config == "ddp-mnist":
        return ddp_mnist(args)
    if args.config == "mxnet-kv":
        if getattr(args, "kv_role_child", False):
            dev = os.environ.get("TONY_KV_WORKER_DEVICE")
            if dev is not None:
                import torch

                if torch.cuda.device_count() > 0:
                    torch.cuda.set_device(int(dev) % torch.cuda.device_count())
            return mxnet_kv_worker(args)
        return mxnet_kv_launch(args, argv)
    raise ValueError(f"unknown --config {args.config!r} (one of {CONFIGS})")
