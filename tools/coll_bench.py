#!/usr/bin/env python3
"""All-reduce / reduce-scatter / all-gather bus bandwidth vs message size: RCCL vs tony_amd's xGMI
peer-memory kernels (parallel/xgmi.py), one process per GPU.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/coll_bench.py

Bus bandwidth follows the nccl-tests convention: all-reduce moves 2 (n-1)/n of the bytes per rank,
reduce-scatter / all-gather (n-1)/n.  Rank 0 prints one markdown table.
"""
from __future__ import annotations

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
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dev = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group("nccl", device_id=dev)
    from tony_amd.parallel.xgmi import XgmiComm

    x = XgmiComm(slot_bytes=256 << 20)
    rows = []
    for mb in (0.0625, 0.25, 1, 4, 16, 64, 128):
        n = int(mb * (1 << 20)) // 2 // (8 * world) * (8 * world)  # bf16 elements, shardable
        t = torch.randn(n, device=dev).to(torch.bfloat16)
        shard = torch.empty(n // world, device=dev, dtype=torch.bfloat16)
        iters = 50 if mb <= 4 else 10
        nbytes = n * 2
        f = (world - 1) / world
        res = {
            "rccl allreduce": (timeit(lambda: dist.all_reduce(t), iters), 2 * f),
            "xgmi allreduce": (timeit(lambda: x.all_reduce(t), iters), 2 * f),
            "rccl reduce_scatter": (timeit(lambda: dist.reduce_scatter_tensor(shard, t), iters), f),
            "xgmi reduce_scatter": (timeit(lambda: x.reduce_scatter(shard, t), iters), f),
            "rccl all_gather": (timeit(lambda: dist.all_gather_into_tensor(t, shard), iters), f),
            "xgmi all_gather": (timeit(lambda: x.all_gather(t, shard), iters), f),
        }
        rows.append((mb, {k: (s * 1e6, nbytes * bw / s / 1e9) for k, (s, bw) in res.items()}))
    x.check_error()
    if rank == 0:
        names = list(rows[0][1])
        print("| MiB | " + " | ".join(f"{k} us (busbw GB/s)" for k in names) + " |")
        print("|---|" + "---|" * len(names))
        for mb, r in rows:
            print(f"| {mb} | " + " | ".join(f"{r[k][0]:.1f} ({r[k][1]:.0f})" for k in names) + " |")
    x.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
