#!/usr/bin/env python3
"""Headline benchmark: Inception-v3 parameter-server training, images/sec (whole node).

BASELINE.json metric: "images/sec (whole node) Inception-v3 TF-PS at 1/2/4/8 MI355X".
One process per GPU (torch.distributed.run, RCCL over xGMI).  Two PS topologies:

``--ps-mode colocated`` (default)
    every process is one TF-PS *worker* and hosts one PS shard (tony_amd/parallel/ps.py).  The
    flat gradient is cut into ~8 MB buckets; as backward completes a bucket, its push (RCCL
    reduce-scatter), apply (fused HIP SGD-momentum on the fp32 master shard) and pull (RCCL
    all-gather) are enqueued on a communication stream while backward continues
    (parallel/buckets.py).
``--ps-mode dedicated``
    the paper topology: rank 0 is the ps task (owns the fp32 variables, runs no model), ranks
    1..N-1 are workers.  Data plane (parallel/ps_plane.py): workers store each bucket's gradient
    straight into the ps GPU's receive window as backward produces it, the ps applies the fused
    optimizer as the rows land and stores the new variables straight into every worker's landing
    window (TONY_PS_PLANE=rccl: reduce / apply / broadcast per bucket instead).  Images/sec counts
    the N-1 workers' images only.  ``--ps-async``: TF's default asynchronous PS (each worker push
    applied on its own as it lands; the headline and the default are synchronous).

Compute is bf16 NHWC with the tony_amd HIP kernels (fused BN+ReLU, MFMA implicit-GEMM convs, fused
heads, fused softmax-xent, fused optimizer); the step is issued eagerly (weight gradients on a side
stream) or replayed as a HIP graph, whichever measured faster in setup (``--mode auto``).
``--dtype fp32`` runs the reference-precision row (TF's Inception-v3 PS job is fp32): fp32
activations, variables and pushed gradients, each conv / GEMM product as an x3 split over the bf16
MFMA kernels (ops/x3.py); ``--stock --dtype fp32``: the stock MIOpen / hipBLASLt fp32 comparator.
``--grad-dtype fp32`` keeps bf16 compute but pushes and sums fp32 gradients.

Data is synthetic (ImageNet-shaped 299x299x3 images, random labels) and weights are random-init --
no network access for datasets / checkpoints.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--ps-mode M] [--dtype D]
       N>1 under torch.distributed.run (WORLD_SIZE set): one rank per GPU, as the driver launches it;
       N>1 without it: bench.py starts ``python -m torch.distributed.run --nproc-per-node N bench.py ...``
       as a child process (never an exec), relays rank 0's JSON line and exits with the child's code.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (weak scaling; default 128, mxnet-kv 1024 rows per worker)")
    ap.add_argument("--mode", default="auto", choices=["auto", "graph", "eager"],
                    help="graph: replay the step as one HIP graph; eager: launch kernels from Python (weight "
                         "gradients overlap the data-gradient chain on a second stream); auto: time both in setup")
    ap.add_argument("--no-graph", action="store_true", help="same as --mode eager")
    ap.add_argument("--ps-mode", default="colocated", choices=["colocated", "dedicated"],
                    help="colocated: one PS shard per GPU; dedicated: rank 0 = the ps task, the rest are workers")
    ap.add_argument("--ps-async", action="store_true",
                    help="--ps-mode dedicated: TF's default asynchronous PS (each worker push applied on its own on "
                         "arrival, the reference mnist_distributed.py example's mode); the headline runs sync")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute dtype; fp32 = the reference-precision row (x3-split MFMA products, fp32 variables)")
    ap.add_argument("--grad-dtype", default=None, choices=["bf16", "fp32"],
                    help="dtype of the pushed / summed gradients (default: the compute dtype)")
    ap.add_argument("--bucket-mb", type=float, default=None, help="gradient bucket size (default 8 MB)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="push/apply/pull every bucket after backward instead of during it")
    ap.add_argument("--stock", action="store_true",
                    help="comparator: stock nn.BatchNorm2d+ReLU / MIOpen convs / torch loss (not the headline)")
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    ap.add_argument("--optimizer", default="sgd")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps (for rocprof)")
    ap.add_argument("--no-wgrad-stream", action="store_true",
                    help="serial backward (no weight gradients on a second stream)")
    ap.add_argument("--no-branch-streams", action="store_true",
                    help="Inception branches on one stream (branch streams are on by default; TONY_BRANCH_STREAMS=0 "
                         "also turns them off)")
    ap.add_argument("--tune-cache", default=None,
                    help="JSON of kernel-choice decisions: loaded when it exists (no autotuning for those "
                         "shapes), written after setup otherwise (reproducible profiles, faster startup)")
    ap.add_argument("--collective", default=None, choices=["rccl", "hip"],
                    help="gradient push / pull collectives: RCCL (default) or tony_amd's xGMI peer-memory "
                         "kernels (csrc/xgmi.hip); sets TONY_COLLECTIVE")
    ap.add_argument("--fp32-row", type=int, default=1,
                    help="N=1 bf16 runs: also time the reference-precision (x3 fp32) step in a child process and "
                         "report it as the record's fp32_row (0: skip)")
    ap.add_argument("--fp32-steps", type=int, default=10)
    ap.add_argument("--fp32-warmup", type=int, default=3)
    ap.add_argument("--no-miopen-find", action="store_true",
                    help="MIOpen immediate mode instead of find (faster startup, slower non-1x1 convs)")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="N>1 without torch.distributed.run: print the self-launch argv / env as JSON and exit")
    ap.add_argument("--config", default="inception-ps",
                    choices=["inception-ps", "hvd-resnet50", "ddp-mnist", "mxnet-kv"],
                    help="which BASELINE.json config to measure: the Inception-v3 PS headline (default) or "
                         "one of the others (tony_amd/bench_configs.py), each one JSON line")
    ap.add_argument("--kvstore", default="dist_sync", help="mxnet-kv: kvstore type (BASELINE: dist_sync)")
    ap.add_argument("--kv-device", default="auto", choices=["auto", "cuda", "cpu"],
                    help="mxnet-kv: where the workers' tensors live (cuda: the GPU payload plane)")
    ap.add_argument("--kv-role-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-bind", action="store_true",
                    help="N>1: leave CPU affinity alone (default: each rank on its GPU's NUMA node CPUs)")
    a = ap.parse_args(argv)
    if a.ps_async and a.ps_mode != "dedicated":
        ap.error("--ps-async needs --ps-mode dedicated (the colocated shards apply synchronously)")
    if a.batch is None:
        a.batch = {"mxnet-kv": 1024}.get(a.config, 128)
    return a


def fail(msg: str, code: int = 4) -> int:
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)
    return code


class _PSOnly:
    """The dedicated ps rank's step: no model.  On the xGMI plane (default) it launches the apply
    kernels that sum the workers' gradient rows as they land in its receive windows and store the new
    variables into every worker's landing window; on the RCCL plane (TONY_PS_PLANE=rccl) it runs the
    bucketed reduce -> apply -> broadcast in the workers' collective order."""

    def __init__(self, ps, dev):
        self.ps = ps
        self.use_graph = False
        self.warmup_eager = 1
        self.host_fwd_s = self.host_bwd_s = 0.0
        self.phase_events = None
        self._zero = torch.zeros((), device=dev)

    def step(self, x, y):  # noqa: ARG002 - the ps runs no model
        self.ps.begin_step(overlap=False)
        self.ps.step()
        return self._zero

    def enable_phase_timing(self):
        pass

    def phase_ms(self):
        return (0.0, 0.0, 0.0)


def diagnose(world: int, rank: int, dev, backend: str, shared_ok: bool) -> dict:
    """N>1 self-checks for the driver's scaling run: one distinct GPU per rank over RCCL.  Returns
    what was found (printed by rank 0); raises SystemExit on a fallback the run must not hide."""
    info = {"backend": backend, "world_size": dist.get_world_size()}
    try:
        info["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
    except Exception:  # noqa: BLE001 - informational
        info["rccl_version"] = None
    p = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "device": dev.index, "bdf": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
          "uuid": str(getattr(p, "uuid", ""))}
    allp = [None] * world
    dist.all_gather_object(allp, me)
    info["devices"] = [a["bdf"] for a in allp]
    # RCCL's transport per rank (P2P over xGMI vs SHM / NET fallbacks), from its INIT,P2P debug log:
    # the channels of the ring/tree are connected by the collectives above
    tr = _rccl_transport()
    allt = [None] * world
    dist.all_gather_object(allt, tr)
    info["transport"] = allt
    if len({a["bdf"] for a in allp}) != world and not shared_ok:
        raise SystemExit(fail(f"ranks share a GPU ({info['devices']}): each rank must own one device"))
    if backend != "nccl" and not shared_ok:
        raise SystemExit(fail(f"process group backend is {backend!r}, not RCCL"))
    return info


_RCCL_LOG = [None]


def _rccl_debug_env(world: int) -> None:
    """Ask RCCL for its INIT,P2P log in a private file (unless the user set NCCL_DEBUG themselves)."""
    if world > 1 and "NCCL_DEBUG" not in os.environ:
        path = f"/tmp/tony_rccl_{os.getpid()}.log"
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,P2P", NCCL_DEBUG_FILE=path)
        _RCCL_LOG[0] = path


def _rccl_transport() -> dict:
    """{transport: channel connections} parsed from RCCL's "... via P2P/IPC" lines (None: no log)."""
    path = _RCCL_LOG[0]
    if path is None or not os.path.exists(path):
        return {}
    out = {}
    with open(path, errors="replace") as f:
        for line in f:
            if " via " not in line:
                continue
            kind = line.split(" via ", 1)[1].split()[0] if line.split(" via ", 1)[1].split() else "?"
            out[kind] = out.get(kind, 0) + 1
    return out


def _heartbeat(t0: float, every_s: float = 45.0) -> None:
    """Progress line while setup runs silently for minutes (MIOpen find, first-step autotuning):
    the GPU-box runner treats a command that stops writing for 3 minutes as hung."""
    import threading

    def beat():
        while True:
            time.sleep(every_s)
            print(f"[bench] alive t={time.perf_counter() - t0:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, name="bench-heartbeat", daemon=True).start()


def bind_rank_cpus():
    """N>1 under torch.distributed.run: pin this rank (and the threads it starts) to CPUs of its GPU's NUMA
    node, split among the local ranks that share the node (gpu/inventory.rank_cpus -- the coordinator's slot
    allocator does the same for launcher tasks).  Runs before any GPU call.  Returns the CPU list (None:
    one rank, a shared-GPU rehearsal, or no NUMA information)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or "TONY_BENCH_DEVICE" in os.environ or not hasattr(os, "sched_setaffinity"):
        return None
    local = int(os.environ.get("LOCAL_RANK", "0"))
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    try:
        from tony_amd.gpu.inventory import rank_cpus

        vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
        kfd = [int(v) for v in vis.split(",") if v.strip()] if vis else list(range(lws))
        if len(kfd) < lws:
            return None
        cpus = rank_cpus(kfd[local], kfd[:lws])
        if cpus:
            os.sched_setaffinity(0, cpus)
        return cpus or None
    except Exception as e:  # noqa: BLE001 - placement is an optimisation, never a failure
        print(f"[bench] rank {local}: CPU binding skipped ({e})", file=sys.stderr, flush=True)
        return None


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch_cmd(argv, n: int, port: int):
    """argv / env of the child that runs ``bench.py --gpus N`` as N ranks, one per GPU (the driver's
    own form: torch.distributed.run, 127.0.0.1 rendezvous)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
    cmd += [a for a in argv if a != "--launch-dry-run"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC: RCCL / tensor sharing across ranks
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return cmd, env


def self_launch(args, argv) -> int:
    """``python bench.py --gpus N`` (N > 1) with no torch.distributed.run around it.  Runs before
    anything touches the GPU in this process, and starts the launcher as a CHILD (an exec from a
    process that initialised the GPU is forbidden on the pool): the ranks inherit stdout, so rank 0's
    JSON line is the one this command prints; the exit code is the launcher's."""
    import signal
    import subprocess

    cmd, env = self_launch_cmd(argv, args.gpus, _free_port())
    if args.launch_dry_run:
        print(json.dumps({"self_launch": cmd, "env": {k: env[k] for k in ("HSA_ENABLE_IPC_MODE_LEGACY",)}}))
        return 0
    n_dev = torch.cuda.device_count()  # counts devices without initialising HIP in this process
    if n_dev < args.gpus and "TONY_BENCH_DEVICE" not in os.environ:  # (rehearsal: ranks share one GPU)
        return fail(f"--gpus {args.gpus} but this node shows {n_dev} GPU(s)", 2)
    print(f"[bench] self-launch: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, env=env, start_new_session=True)

    def forward(sig, _frame):  # the driver's timeout / ^C reaches every rank
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            pass

    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        return p.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.collective:
        os.environ["TONY_COLLECTIVE"] = args.collective
    if args.config == "mxnet-kv":  # scheduler + server + N workers (its own launcher, bench_configs.py)
        from tony_amd import bench_configs

        return bench_configs.run(args, argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args, argv)
    cpus = None if args.no_bind else bind_rank_cpus()  # before any GPU call in this process
    if args.config != "inception-ps":
        from tony_amd import bench_configs

        return bench_configs.run(args, argv)
    if int(os.environ.get("RANK", "0")) == 0:
        _heartbeat(time.perf_counter())
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        return fail(f"--gpus {args.gpus} but WORLD_SIZE={world}: N>1 must be launched with torch.distributed.run "
                    f"--nproc-per-node N", 2)
    if args.ps_mode == "dedicated" and world < 2:
        return fail("--ps-mode dedicated needs >= 2 ranks (1 ps + workers)", 2)
    # test hooks for rehearsing the multi-rank path on a one-GPU box: several ranks on one device
    # over gloo (TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("TONY_BENCH_BACKEND", "nccl")
    rehearsal = "TONY_BENCH_BACKEND" in os.environ or "TONY_BENCH_DEVICE" in os.environ
    dev_index = int(os.environ.get("TONY_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    diag = {}
    if world > 1 and backend == "nccl":
        _rccl_debug_env(world)
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        diag = diagnose(world, rank, dev, dist.get_backend(), rehearsal)

    from tony_amd.ops import cross_entropy, tune
    from tony_amd.parallel import collectives as coll
    from tony_amd.parallel.collectives import max_over_ranks
    from tony_amd.parallel.ps import ParameterServer
    from tony_amd.parallel.trainer import Trainer

    torch.backends.cudnn.benchmark = not args.no_miopen_find  # MIOpen find for the MIOpen convs
    fp32 = args.dtype == "fp32"
    dtype = torch.float32 if fp32 else torch.bfloat16
    grad_dtype = {"bf16": torch.bfloat16, "fp32": torch.float32, None: dtype}[args.grad_dtype]
    # fp32 (the reference's precision): Inception-v3 on the x3-split kernels (ops/x3.py: fp32 tensors,
    # bf16-MFMA products of hi/lo operand planes); --stock: the stock MIOpen / hipBLASLt comparator
    x3 = fp32 and not args.stock and args.model == "inception_v3"
    fused = not (args.stock or fp32)
    if args.model == "inception_v3":
        from tony_amd.models.inception_v3 import inception_v3
        model = inception_v3(fused=fused, seed=0, precision="fp32" if x3 else "bf16")
        res, aux_w = 299, 0.4
    else:
        from tony_amd.models.resnet import resnet50
        model = resnet50(fused=fused, seed=0)
        res, aux_w = 224, 0.0
    model = model.to(dev).to(memory_format=torch.channels_last)
    model.train()
    ps_kw = {} if args.bucket_mb is None else {"bucket_mb": args.bucket_mb}
    if os.environ.get("TONY_BUCKETED_SINGLE", "0") == "1":
        # one rank: the bucket engine applies each bucket as soon as backward has written it (the
        # optimizer overlaps the backward tail) instead of one apply after the join
        ps_kw["bucketed_single"] = True
    ps = ParameterServer(model, optimizer=args.optimizer, lr=0.045 if args.model == "inception_v3" else 0.1,
                         momentum=0.9, weight_decay=4e-5, mode=args.ps_mode, ps_ranks=(0,), dtype=dtype, device=dev,
                         wire_dtype=grad_dtype, sync=not args.ps_async, **ps_kw)
    if args.ps_async and ps.plane is None:
        return fail("--ps-async needs the xGMI PS data plane (GPU ranks)", 2)
    n_workers = len(ps.worker_ranks)

    if fused or x3:
        xent = cross_entropy
    else:
        def xent(logits, y):
            return torch.nn.functional.cross_entropy(logits.float(), y)

    def loss_fn(out, y):
        if isinstance(out, tuple):
            logits, aux = out
            return xent(logits, y) + aux_w * xent(aux, y)
        return xent(out, y)

    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.randn((args.batch, 3, res, res), generator=g, device=dev, dtype=torch.float32)
    x = x.to(dtype).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), generator=g, device=dev)

    tune_loaded = 0
    if args.tune_cache and os.path.exists(args.tune_cache):
        tune_loaded = tune.load(args.tune_cache)
    mode = "eager" if args.no_graph else args.mode
    if mode == "auto" and world > 1 and os.environ.get("TONY_BENCH_AUTO_PLAN", "1") == "0":
        # escape hatch: eager at N > 1 without timing the native plan (auto times both by default; the
        # plan replays per-bucket segments so the PS collectives still overlap backward)
        mode = "eager"
    if ps.is_worker:
        trainer = Trainer(model, ps, loss_fn, use_graph=mode != "eager", overlap_wgrad=not args.no_wgrad_stream,
                          branch_streams=not args.no_branch_streams, overlap_comm=not args.no_overlap)
    else:
        trainer = _PSOnly(ps, dev)
    t_w = time.perf_counter()
    setup = {}
    if mode == "auto":
        # Setup (untimed, before the W warmup steps): the first step autotunes every conv / GEMM shape,
        # then eager steps and graph replays are timed and the faster way of issuing the step is
        # kept -- eager launches overlap the weight gradients with the data-gradient chain on a second
        # stream and the bucketed PS communication with backward, which a replayed graph does not.
        issue = [0.0]  # host seconds spent inside trainer.step over the last window

        def timed(n):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            issue[0] = 0.0
            for _ in range(n):
                th = time.perf_counter()
                trainer.step(x, y)
                issue[0] += time.perf_counter() - th
            torch.cuda.synchronize()
            return max_over_ranks(time.perf_counter() - t, device=dev) / n

        def window(graph: bool, n: int = 4):
            trainer.use_graph = graph and ps.is_worker
            w = timed(n)
            return w, issue[0] / n

        for _ in range(trainer.warmup_eager):
            trainer.step(x, y)
        trainer.use_graph = False
        timed(2)  # the warm-up steps ran on a side stream: let the allocator fill this stream's pool
        trainer.use_graph = ps.is_worker
        trainer.step(x, y)  # capture
        # alternating windows (eager, plan, eager, plan, ...): a box's slow minute hits both modes alike;
        # best window per mode
        ew, gw, eh = [], [], []
        for _ in range(3):
            w, h = window(False)
            ew.append(w)
            eh.append(h)
            gw.append(window(True)[0])
        setup["eager_ms"] = round(1000 * min(ew), 3)
        setup["graph_ms"] = round(1000 * min(gw), 3)
        # host issue of an eager step: near the GPU time, a host slowed by other work on the machine stalls
        # the GPU (an eager run timed at 15.3 ms/step after its setup measured 13.4,
        # profiles/r4_bench_host_bound_eager.md); the plan issues a step in ~2.5 ms
        setup["eager_host_ms"] = round(1000 * min(eh), 3)
        eager_host_bound = setup["eager_host_ms"] > EAGER_HOST_BOUND * setup["eager_ms"]
        # one rank: the faster schedule wins; eager needs a margin only when its issue is near host-bound.
        # Several ranks: a replay's bucket collectives interleave with its segments, the plan must win.
        if world == 1:
            mode = "graph" if (setup["graph_ms"] <= setup["eager_ms"] * (PLAN_TIE if eager_host_bound else 1.0)) \
                else "eager"
        else:
            mode = "graph" if setup["graph_ms"] <= setup["eager_ms"] else "eager"
        setup["eager_host_bound"] = eager_host_bound
        trainer.use_graph = mode == "graph" and ps.is_worker
        if rank == 0:
            print(f"[bench] setup {time.perf_counter() - t_w:.1f}s: {setup} -> {mode}", file=sys.stderr, flush=True)
    loss = None
    for i in range(args.warmup):
        loss = trainer.step(x, y)
        if rank == 0:
            torch.cuda.synchronize()
            print(f"[bench] warmup {i + 1}/{args.warmup} t={time.perf_counter() - t_w:.1f}s", file=sys.stderr,
                  flush=True)
    torch.cuda.synchronize()
    # every rank decides together: a rank that stopped alone would leave the others in a collective
    bad = torch.tensor([0.0 if loss is None or torch.isfinite(loss).all() else 1.0], device=dev)
    if world > 1:
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
    if bad.item():
        return fail(f"non-finite loss after warmup on some rank (rank {rank}: {loss.float().item()})", 3)

    if args.tune_cache and not tune_loaded and rank == 0:  # every shape has been tuned by now
        n_saved = tune.save(args.tune_cache)
        print(f"[bench] saved {n_saved} kernel-choice decisions to {args.tune_cache}", file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0  # host time spent issuing the steps (the GPU must stay the bottleneck in eager mode)
    for _ in range(args.steps):
        th = time.perf_counter()
        loss = trainer.step(x, y)
        host += time.perf_counter() - th
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # untimed: GPU time per step with the host far ahead (a spin kernel holds the GPU while the host
    # enqueues the steps): equal to ms_per_step when the step is GPU-bound, lower when host launch
    # overhead leaves the GPU waiting
    gpu_ahead = host_free = None
    if world == 1 and (trainer.use_graph is False or getattr(trainer, "plan", None) is not None):
        n_ahead = 6
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e6 * 16 * n_ahead))  # ~2.4 GHz x 16 ms x n_ahead
        e0.record()
        th = time.perf_counter()
        for _ in range(n_ahead):
            loss = trainer.step(x, y)
        host_free = (time.perf_counter() - th) / n_ahead  # issue cost while the GPU is still spinning
        e1.record()
        e1.synchronize()
        gpu_ahead = round(e0.elapsed_time(e1) / n_ahead, 3)
    # untimed: one eager step with GPU events at the phase boundaries (fwd / bwd / exposed PS tail)
    phases = None
    was_graph = trainer.use_graph
    trainer.use_graph = False
    trainer.enable_phase_timing()
    trainer.step(x, y)
    phases = [max_over_ranks(v, device=dev) for v in trainer.phase_ms()]
    trainer.phase_events = None
    trainer.use_graph = was_graph
    for _ in range(args.profile_steps):
        trainer.step(x, y)
    torch.cuda.synchronize()

    elapsed = max_over_ranks(elapsed, device=dev)
    # the dedicated ps rank runs no model: report a worker's loss
    final_loss = max_over_ranks(float(loss.float().item()) if ps.is_worker else float("-inf"), device=dev)
    fallbacks = coll.fallback_count()
    # this rank's engine: in --ps-mode dedicated rank 0 is the ps (no model, no step plan), so the
    # record carries the first worker's engine / host statistics (gathered from every rank)
    eng = {
        "hip_graph": mode == "graph" and getattr(trainer, "replay_kind", None) == "graph",
        # plan: the step captured once and re-issued natively (ops/plan.py, csrc/plan.hip)
        "step_mode": "plan" if mode == "graph" and getattr(trainer, "replay_kind", None) == "plan" else mode,
        "plan_stats": trainer.plan.stats if getattr(trainer, "plan", None) is not None else None,
        "plan_error": getattr(trainer, "plan_error", None),
        "buckets_overlapped_with_backward": ps.overlapped_buckets,
        "host_ms_per_step": round(1000.0 * host / args.steps, 3),
        "gpu_ms_per_step_host_ahead": gpu_ahead,
        "host_ms_per_step_unblocked": None if host_free is None else round(1000.0 * host_free, 3),
        "host_fwd_bwd_ms_last_eager_step": [round(1000.0 * trainer.host_fwd_s, 3), round(1000.0 * trainer.host_bwd_s, 3)],
        "conv_impl": _conv_impl_counts(),
    }
    # per rank: host issue time per timed step, the setup's eager host time / host-bound verdict, its CPUs
    mine = {"rank": rank, "host_ms_per_step": eng["host_ms_per_step"],
            "eager_host_ms": setup.get("eager_host_ms"), "eager_host_bound": setup.get("eager_host_bound"),
            "cpus": None if cpus is None else f"{len(cpus)} ({cpus[0]}-{cpus[-1]})"}
    engines, ranks_host = [eng], [mine]
    if world > 1:
        engines = [None] * world
        dist.all_gather_object(engines, eng)
        ranks_host = [None] * world
        dist.all_gather_object(ranks_host, mine)
    eng_rank = ps.worker_ranks[0] if ps.worker_ranks else 0
    eng = dict(engines[eng_rank], engine_of_rank=eng_rank)
    fp32_row = None
    if args.fp32_row and args.dtype == "bf16" and args.model == "inception_v3" and not args.stock:
        if world == 1:
            # reference precision under the same clock discipline: the x3 fp32 step in a child process
            fp32_row = _fp32_row(args)
        else:
            # N ranks: the x3 fp32 step in-process after the bf16 timed region, on the same process group
            # (no child launch: the ranks and their RCCL communicator are already up)
            fp32_row = _fp32_row_inprocess(args, world, rank, dev)
    if rank == 0:
        imgs = args.batch * n_workers * args.steps
        value = imgs / elapsed
        if args.ps_mode == "colocated":
            par = f"ps-colocated-sharded dp{world} (1 PS shard + 1 worker per GPU, sync)"
        else:
            par = (f"ps-dedicated 1 ps + {n_workers} workers ({'sync' if ps.sync else 'async'}, {ps.plane_kind} "
                   "data plane)")
        rec = {
            "metric": "images/sec (whole node) Inception-v3 TF-PS" if args.model == "inception_v3"
            else "images/sec (whole node) ResNet-50",
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": f"synthetic ImageNet-shaped {res}x{res}x3 batches, random-init weights",
            "config": {
                "model": args.model,
                "global_batch": args.batch * n_workers,
                "per_gpu_batch": args.batch,
                "seq_len": None,
                "image_size": res,
                "parallelism": par,
                "ps_mode": args.ps_mode,
                "workers": n_workers,
                "grad_dtype": "fp32" if grad_dtype == torch.float32 else "bf16",
                "variables": f"fp32 master on the PS, {args.dtype} compute copy",
                "optimizer": "fused SGD-momentum (HIP)" if args.optimizer == "sgd" else args.optimizer,
                **eng,
                "mode_setup_ms": setup or None,
                "tune_cache_loaded": tune_loaded,
                "wgrad_stream": not args.no_wgrad_stream,
                "branch_streams": _branch_streams_on(args),
                "grad_buckets": len(ps.buckets),
                "phase_ms_eager_step_max_over_ranks":
                    dict(zip(("forward", "backward", "exposed_ps_push_apply_pull"), [round(v, 3) for v in phases])),
                "kernels": "tony_amd HIP" if fused else (
                    "tony_amd HIP, fp32 via x3-split bf16 MFMA products (ops/x3.py)" if x3
                    else "stock PyTorch-ROCm (MIOpen / hipBLASLt)"),
                "collective": "hip-xgmi" if os.environ.get("TONY_COLLECTIVE", "rccl").lower() in ("hip", "xgmi")
                else ("rccl" if dist.is_initialized() and dist.get_backend() == "nccl" else None),
                "collective_fallbacks": fallbacks,
                # init-time canaries of the hand data planes against RCCL (None: that plane unused)
                "data_plane_verified": coll.data_plane_status(),
                "dist": diag or None,
                "ranks_host": ranks_host if world > 1 else None,
                "ps_sync": ("synchronous: every step sums all workers' gradients before the apply (TonY's "
                            "mnist_distributed.py example trains asynchronously; a sync step does at least the same "
                            "work, and bench.py --ps-mode dedicated --ps-async / jobs/inception_ps.py --async run "
                            "the async form)") if ps.sync else
                           ("asynchronous: each worker's push is applied on its own as it lands and only that "
                            "worker's variables are refreshed (TF's default PS mode, the reference example's)"),
                "final_loss": round(final_loss, 4),
            },
        }
        if fp32_row is not None:
            # the reference's precision (TF's Inception-v3 PS job is fp32 end to end): same model and
            # batch, fp32 activations / gradients / variables, conv and GEMM products as x3-split
            # bf16 MFMAs (ops/x3.py); timed by its own barrier + synchronize bracket in a child process
            rec["fp32_row"] = fp32_row
        print(json.dumps(rec), flush=True)
    rc = 0
    if os.environ.get("TONY_COLLECTIVE", "rccl").lower() in ("hip", "xgmi") and fallbacks:
        rc = fail(f"TONY_COLLECTIVE=xgmi requested but {fallbacks} collectives fell back to RCCL")
    if ps.plane is not None:
        ps.plane.close()
    if world > 1:
        dist.destroy_process_group()
    return rc


# --mode auto at one rank: the faster of eager and plan; when eager's host issue time per step exceeds
# EAGER_HOST_BOUND x its step time (close to host-bound: a busier host would stall the GPU), eager must
# beat the plan by more than PLAN_TIE (TONY_PLAN_TIE / TONY_EAGER_HOST_BOUND)
PLAN_TIE = float(os.environ.get("TONY_PLAN_TIE", "1.01"))
EAGER_HOST_BOUND = float(os.environ.get("TONY_EAGER_HOST_BOUND", "0.8"))


def _fp32_row(args) -> dict:
    """Run ``bench.py --dtype fp32`` (same model, batch and issue mode) as a child process -- never an
    exec from this GPU-initialised process -- and return its timing as the fp32 row."""
    import subprocess

    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--steps", str(args.fp32_steps),
           "--warmup", str(args.fp32_warmup), "--batch", str(args.batch), "--dtype", "fp32", "--fp32-row", "0",
           "--mode", "eager" if args.no_graph else args.mode]
    env = dict(os.environ)
    env.pop("RANK", None)
    t = time.perf_counter()
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "fp32 child timed out"}
    line = next((ln for ln in reversed(p.stdout.splitlines()) if ln.startswith("{")), None)
    if p.returncode != 0 or line is None:
        tail = (p.stderr or "").strip().splitlines()[-3:]
        return {"error": f"fp32 child rc={p.returncode}: {' | '.join(tail)}"}
    r = json.loads(line)
    c = r.get("config", {})
    return {"value": r["value"], "unit": r["unit"], "ms_per_step": r["ms_per_step"], "steps": r["steps"],
            "warmup": r["warmup"], "dtype": "fp32", "kernels": c.get("kernels"), "step_mode": c.get("step_mode"),
            "final_loss": c.get("final_loss"), "child_wall_s": round(time.perf_counter() - t, 1)}


def _fp32_row_inprocess(args, world: int, rank: int, dev) -> dict:
    """N > 1: the reference-precision step (x3 fp32 Inception-v3, fp32 variables and pushed gradients,
    colocated sharded PS) built and timed in this rank after the bf16 run, on the same process group:
    ``--fp32-warmup`` untimed steps, then ``--fp32-steps`` timed ones bracketed by barrier + synchronize on
    both sides, the max over ranks.  Eager issue (the x3 step is ~2.3x the bf16 one: far from host-bound)."""
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.ops import cross_entropy
    from tony_amd.parallel.collectives import max_over_ranks
    from tony_amd.parallel.ps import ParameterServer
    from tony_amd.parallel.trainer import Trainer

    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    t_all = time.perf_counter()
    try:
        model = inception_v3(fused=False, seed=0, precision="fp32").to(dev).to(memory_format=torch.channels_last)
        model.train()
        ps = ParameterServer(model, optimizer=args.optimizer, lr=0.045, momentum=0.9, weight_decay=4e-5,
                             mode="colocated", ps_ranks=(0,), dtype=torch.float32, device=dev,
                             wire_dtype=torch.float32)

        def loss_fn(out, y):
            logits, aux = out
            return cross_entropy(logits, y) + 0.4 * cross_entropy(aux, y)

        trainer = Trainer(model, ps, loss_fn, use_graph=False, overlap_wgrad=not args.no_wgrad_stream,
                          branch_streams=not args.no_branch_streams, overlap_comm=not args.no_overlap)
        g = torch.Generator(device=dev).manual_seed(4321 + rank)
        x = torch.randn((args.batch, 3, 299, 299), generator=g, device=dev).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (args.batch,), generator=g, device=dev)
        loss = None
        for _ in range(max(1, args.fp32_warmup)):
            loss = trainer.step(x, y)
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.fp32_steps):
            loss = trainer.step(x, y)
        torch.cuda.synchronize(dev)
        dist.barrier()
        el = max_over_ranks(time.perf_counter() - t0, device=dev)
        fin = max_over_ranks(float(loss.float().item()), device=dev)
        if ps.plane is not None:
            ps.plane.close()
    except Exception as e:  # noqa: BLE001 - reported in the record, the bf16 headline stands
        return {"error": f"in-process fp32 step failed on rank {rank}: {type(e).__name__}: {e}"}
    n_workers = len(ps.worker_ranks)
    return {"value": round(args.batch * n_workers * args.fp32_steps / el, 2), "unit": "images/sec",
            "ms_per_step": round(1000.0 * el / args.fp32_steps, 3), "steps": args.fp32_steps,
            "warmup": max(1, args.fp32_warmup), "dtype": "fp32", "n_gpus": world,
            "kernels": "tony_amd HIP, fp32 via x3-split bf16 MFMA products (ops/x3.py)", "step_mode": "eager",
            "parallelism": f"ps-colocated-sharded dp{world} (sync), fp32 variables and gradients",
            "final_loss": round(fin, 4), "timed_in": "same ranks, after the bf16 run",
            "wall_s": round(time.perf_counter() - t_all, 1)}


def _branch_streams_on(args) -> bool:
    from tony_amd.ops import streams

    return streams.BRANCHES_ENABLED and not args.no_branch_streams and not args.no_wgrad_stream


def _conv_impl_counts():
    """How many (pass, shape) conv problems went to tony_amd's kernels vs MIOpen."""
    from tony_amd.ops.conv import choices

    out = {}
    for (pas, *_), impl in choices().items():
        out[f"{pas}:{impl}"] = out.get(f"{pas}:{impl}", 0) + 1
    return out


if __name__ == "__main__":
    sys.exit(main())
