#!/usr/bin/env python3
"""Headline benchmark: Inception-v3 parameter-server training, images/sec (whole node).

BASELINE.json metric: "images/sec (whole node) Inception-v3 TF-PS at 1/2/4/8 MI355X".
One process per GPU (torch.distributed.run), each process is one TF-PS *worker*
and hosts one PS shard (colocated sharded PS, tony_amd/parallel/ps.py):
push = RCCL reduce-scatter of bf16 grads over xGMI, apply = fused HIP SGD-momentum
on the fp32 master shard, pull = RCCL all-gather of bf16 variables.  Compute is
bf16 NHWC with the tony_amd HIP kernels (fused BN+ReLU, MFMA 1x1-conv GEMM,
fused softmax-xent, fused optimizer); the whole step is replayed as a HIP graph.

Data is synthetic (ImageNet-shaped 299x299x3 images, random labels) and weights
are random-init -- no network access for datasets / checkpoints.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       (N>1 is launched by the driver via torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128, help="per-GPU batch (weak scaling)")
    ap.add_argument("--mode", default="auto", choices=["auto", "graph", "eager"],
                    help="graph: replay the step as one HIP graph; eager: launch kernels from Python (weight "
                         "gradients overlap the data-gradient chain on a second stream); auto: time both in setup")
    ap.add_argument("--no-graph", action="store_true", help="same as --mode eager")
    ap.add_argument("--stock", action="store_true",
                    help="comparator: stock nn.BatchNorm2d+ReLU / MIOpen 1x1 / torch loss (not the headline)")
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    ap.add_argument("--optimizer", default="sgd")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps (for rocprof)")
    ap.add_argument("--no-wgrad-stream", action="store_true",
                    help="serial backward (no weight gradients on a second stream)")
    ap.add_argument("--no-branch-streams", action="store_true",
                    help="Inception branches on one stream (branch streams are opt-in: TONY_BRANCH_STREAMS=1)")
    ap.add_argument("--tune-cache", default=None,
                    help="JSON of kernel-choice decisions: loaded when it exists (no autotuning for those "
                         "shapes), written after setup otherwise (reproducible profiles, faster startup)")
    ap.add_argument("--no-miopen-find", action="store_true",
                    help="MIOpen immediate mode instead of find (faster startup, slower non-1x1 convs)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print(f"bench.py: --gpus {args.gpus} must be launched with torch.distributed.run", file=sys.stderr)
            return 2
    # test hooks for rehearsing the multi-rank path on a one-GPU box: several ranks on one device
    # over gloo (TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("TONY_BENCH_BACKEND", "nccl")
    dev_index = int(os.environ.get("TONY_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    from tony_amd.ops import cross_entropy
    from tony_amd.parallel.ps import ParameterServer
    from tony_amd.parallel.trainer import Trainer

    torch.backends.cudnn.benchmark = not args.no_miopen_find  # MIOpen find for the remaining MIOpen convs
    fused = not args.stock
    if args.model == "inception_v3":
        from tony_amd.models.inception_v3 import inception_v3
        model = inception_v3(fused=fused, seed=0)
        res, aux_w = 299, 0.4
    else:
        from tony_amd.models.resnet import resnet50
        model = resnet50(fused=fused, seed=0)
        res, aux_w = 224, 0.0
    model = model.to(dev).to(memory_format=torch.channels_last)
    model.train()
    ps = ParameterServer(model, optimizer=args.optimizer, lr=0.045 if args.model == "inception_v3" else 0.1,
                         momentum=0.9, weight_decay=4e-5, mode="colocated", device=dev)

    if fused:
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
    x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), generator=g, device=dev)

    from tony_amd.parallel.collectives import max_over_ranks

    from tony_amd.ops import tune

    tune_loaded = 0
    if args.tune_cache and os.path.exists(args.tune_cache):
        tune_loaded = tune.load(args.tune_cache)
    mode = "eager" if args.no_graph else args.mode
    trainer = Trainer(model, ps, loss_fn, use_graph=mode != "eager", overlap_wgrad=not args.no_wgrad_stream,
                      branch_streams=not args.no_branch_streams)
    t_w = time.perf_counter()
    setup = {}
    if mode == "auto":
        # Setup (untimed, before the W warmup steps): the first step autotunes every conv / GEMM shape,
        # then 3 eager steps and 3 graph replays are timed and the faster way of issuing the step is
        # kept -- eager launches overlap the weight gradients with the data-gradient chain on a second
        # stream, which the HIP-graph runtime's own multi-queue scheduling of the same DAG does not.
        def timed(n):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(n):
                trainer.step(x, y)
            torch.cuda.synchronize()
            return max_over_ranks(time.perf_counter() - t, device=dev) / n

        for _ in range(trainer.warmup_eager):
            trainer.step(x, y)
        trainer.use_graph = False
        timed(2)  # the warm-up steps ran on a side stream: let the allocator fill this stream's pool
        # best of two windows per mode: one host hiccup must not decide the mode for the whole run
        setup["eager_ms"] = round(1000 * min(timed(4), timed(4)), 3)
        trainer.use_graph = True
        trainer.step(x, y)  # capture
        setup["graph_ms"] = round(1000 * min(timed(4), timed(4)), 3)
        mode = "graph" if setup["graph_ms"] <= setup["eager_ms"] else "eager"
        trainer.use_graph = mode == "graph"
        if rank == 0:
            print(f"[bench] setup {time.perf_counter() - t_w:.1f}s: {setup} -> {mode}", file=sys.stderr, flush=True)
    for i in range(args.warmup):
        loss = trainer.step(x, y)
        if rank == 0:
            torch.cuda.synchronize()
            print(f"[bench] warmup {i + 1}/{args.warmup} t={time.perf_counter() - t_w:.1f}s", file=sys.stderr,
                  flush=True)
    torch.cuda.synchronize()
    if not torch.isfinite(loss).all():
        print(f"bench.py: non-finite loss after warmup: {loss.item()}", file=sys.stderr)
        return 3

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
    for _ in range(args.profile_steps):
        trainer.step(x, y)
    torch.cuda.synchronize()

    elapsed = max_over_ranks(elapsed, device=dev)
    final_loss = float(loss.float().item())
    if rank == 0:
        imgs = args.batch * world * args.steps
        value = imgs / elapsed
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
            "dtype": "bf16",
            "data": f"synthetic ImageNet-shaped {res}x{res}x3 batches, random-init weights",
            "config": {
                "model": args.model,
                "global_batch": args.batch * world,
                "per_gpu_batch": args.batch,
                "seq_len": None,
                "image_size": res,
                "parallelism": f"ps-colocated-sharded dp{world} (1 PS shard + 1 worker per GPU, sync)",
                "optimizer": "fused SGD-momentum (HIP)" if args.optimizer == "sgd" else args.optimizer,
                "hip_graph": mode == "graph",
                "step_mode": mode,
                "mode_setup_ms": setup or None,
                "tune_cache_loaded": tune_loaded,
                "wgrad_stream": not args.no_wgrad_stream,
                "branch_streams": _branch_streams_on(args),
                "host_ms_per_step": round(1000.0 * host / args.steps, 3),
                "host_fwd_bwd_ms_last_eager_step": [round(1000.0 * trainer.host_fwd_s, 3),
                                                    round(1000.0 * trainer.host_bwd_s, 3)],
                "kernels": "stock-comparator" if args.stock else "tony_amd HIP",
                "conv_impl": _conv_impl_counts(),
                "grad_buckets": len(ps.buckets),
                "buckets_overlapped_with_backward": ps.overlapped_buckets,
                "final_loss": round(final_loss, 4),
            },
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def _branch_streams_on(args) -> bool:
    from tony_amd.ops import streams

    return streams.BRANCHES_ENABLED and not args.no_branch_streams and not args.no_wgrad_stream


def _conv_impl_counts():
    """How many (pass, shape) conv problems the autotuner gave to tony_amd's kernels vs MIOpen."""
    from tony_amd.ops.conv import choices

    out = {}
    for (pas, *_), impl in choices().items():
        out[f"{pas}:{impl}"] = out.get(f"{pas}:{impl}", 0) + 1
    return out


if __name__ == "__main__":
    sys.exit(main())
