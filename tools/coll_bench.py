#!/usr/bin/env python3
"""All-reduce / reduce-scatter / all-gather bus bandwidth vs message size: RCCL vs tony_amd's xGMI
peer-memory kernels (parallel/xgmi.py), one process per GPU.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/coll_bench.py \
        [--json gpurun_out/coll.json] [--max-mb 128]

Bus bandwidth follows the nccl-tests convention: all-reduce moves 2 (n-1)/n of the bytes per rank,
reduce-scatter / all-gather (n-1)/n.  Every result is checked against the RCCL (or, in a gloo
rehearsal, a host-computed) reference before it is timed.  Rank 0 prints one markdown table and,
with --json, writes the rows as JSON.

One-GPU rehearsal (several ranks sharing device 0, gloo for the handshake, xGMI kernels only):
    TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nproc-per-node 2 \
        --master-addr 127.0.0.1 tools/coll_bench.py --max-mb 16
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--max-mb", type=float, default=128)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    backend = os.environ.get("TONY_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(int(os.environ.get("TONY_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
    dev = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
    rccl = backend == "nccl"
    from tony_amd.parallel.xgmi import XgmiComm

    x = XgmiComm(slot_bytes=256 << 20)
    rows = []
    sizes = [mb for mb in (0.0625, 0.25, 1, 4, 16, 54, 64, 128) if mb <= args.max_mb]
    for mb in sizes:
        n = int(mb * (1 << 20)) // 2 // (8 * world) * (8 * world)  # bf16 elements, shardable
        g = torch.Generator(device=dev).manual_seed(rank)
        t = torch.randn(n, device=dev, generator=g).to(torch.bfloat16)
        shard = torch.empty(n // world, device=dev, dtype=torch.bfloat16)
        full = torch.empty(n, device=dev, dtype=torch.bfloat16)
        # correctness first: xGMI vs an fp32 reference of the same reduction
        ref = t.float().clone()
        if rccl:
            dist.all_reduce(ref)
        else:
            parts = [torch.empty_like(ref) for _ in range(world)]
            dist.all_gather(parts, ref)
            ref = sum(parts)
        got = t.clone()
        x.all_reduce(got)
        x.reduce_scatter(shard, t)
        x.all_gather(full, shard)
        ok = bool(torch.allclose(got.float(), ref, rtol=2e-2, atol=5e-2 * world)
                  and torch.allclose(full.float(), ref, rtol=2e-2, atol=5e-2 * world))
        iters = 50 if mb <= 4 else 10
        nbytes = n * 2
        f = (world - 1) / world
        tt = t.clone()
        res = {
            "xgmi allreduce": (timeit(lambda: x.all_reduce(tt), iters), 2 * f),
            "xgmi reduce_scatter": (timeit(lambda: x.reduce_scatter(shard, t), iters), f),
            "xgmi all_gather": (timeit(lambda: x.all_gather(full, shard), iters), f),
        }
        if rccl:
            res.update({
                "rccl allreduce": (timeit(lambda: dist.all_reduce(tt), iters), 2 * f),
                "rccl reduce_scatter": (timeit(lambda: dist.reduce_scatter_tensor(shard, t), iters), f),
                "rccl all_gather": (timeit(lambda: dist.all_gather_into_tensor(full, shard), iters), f),
            })
        rows.append({"MiB": mb, "bytes": nbytes, "correct": ok,
                     **{k: {"us": round(s * 1e6, 1), "busbw_GBps": round(nbytes * bw / s / 1e9, 1)}
                        for k, (s, bw) in res.items()}})
    x.check_error()
    if rank == 0:
        names = [k for k in rows[0] if isinstance(rows[0][k], dict)]
        print(f"world {world}, backend {backend}, one GPU per rank: {rccl}")
        print("| MiB | ok | " + " | ".join(f"{k} us (busbw GB/s)" for k in names) + " |")
        print("|---|---|" + "---|" * len(names))
        for r in rows:
            print(f"| {r['MiB']} | {r['correct']} | " + " | ".join(
                f"{r[k]['us']} ({r[k]['busbw_GBps']})" for k in names) + " |")
        if args.json:
            with open(args.json, "w") as fh:
                json.dump({"world": world, "backend": backend, "rows": rows}, fh, indent=1)
    x.close()
    dist.destroy_process_group()
    return 0 if all(r["correct"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
