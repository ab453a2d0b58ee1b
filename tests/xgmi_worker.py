"""Rank body for tests/test_xgmi_gpu.py (importable by spawned processes)."""
import os

import torch
import torch.distributed as dist

import gpu_ranks


def run(rank, world, port, q, skip=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dev, _ = gpu_ranks.init(rank, world)  # own GPU per rank over RCCL, or all on the box's one GPU
        from tony_amd.parallel.xgmi import XgmiComm, XgmiError

        comm = XgmiComm(slot_bytes=1 << 20, oneshot_max_bytes=64 << 10, blocks=8)
        res = {}
        for dtype in (torch.float32, torch.bfloat16):
            # one-shot, two-shot, odd size (two-shot pieces + a one-shot tail), multi-piece
            for n in (1024, 40960, 100040, 3 * (1 << 20) // 4 + 4096):
                t = torch.full((n,), float(rank + 1), device=dev, dtype=dtype)
                t += torch.arange(n, device=dev, dtype=torch.float32).remainder(7).to(dtype)
                comm.all_reduce(t)
                exp = (torch.arange(n, device=dev, dtype=torch.float32).remainder(7) * world
                       + sum(range(1, world + 1)))
                res[f"ar_{dtype}_{n}"] = bool(torch.allclose(t.float(), exp, rtol=1e-2, atol=1e-2))
            x = torch.arange(world * 2048, device=dev, dtype=dtype) * (rank + 1)
            out = torch.empty(2048, device=dev, dtype=dtype)
            comm.reduce_scatter(out, x)
            base = torch.arange(world * 2048, device=dev, dtype=torch.float32)[rank * 2048:(rank + 1) * 2048]
            res[f"rs_{dtype}"] = bool(torch.allclose(out.float(), base * sum(range(1, world + 1)), rtol=1e-2))
            shard = torch.full((4096,), float(rank), device=dev, dtype=dtype)
            g = torch.empty(world * 4096, device=dev, dtype=dtype)
            comm.all_gather(g, shard)
            res[f"ag_{dtype}"] = bool(torch.equal(g.float().view(world, 4096)[:, 0].cpu(),
                                                  torch.arange(world, dtype=torch.float32)))
            b = torch.full((8192,), float(rank + 10), device=dev, dtype=dtype)
            comm.broadcast(b, src=1)
            res[f"bc_{dtype}"] = bool((b.float() == 11.0).all().item())
            # larger than the 1 MB slot: reduce-scatter / all-gather go in slot-sized pieces
            m = (3 << 20) // 4 // world // 8 * 8 + 8 * 13            # odd piece count, not a slot multiple
            x = (torch.arange(world * m, device=dev, dtype=torch.float32).remainder(5) + rank).to(dtype)
            out = torch.empty(m, device=dev, dtype=dtype)
            comm.reduce_scatter(out, x)
            full = sum((torch.arange(world * m, device=dev, dtype=torch.float32).remainder(5) + r) for r in range(world))
            res[f"rs_big_{dtype}"] = bool(torch.allclose(out.float(), full[rank * m:(rank + 1) * m], rtol=1e-2))
            shard = (torch.arange(m, device=dev, dtype=torch.float32).remainder(3) + 10 * rank).to(dtype)
            g = torch.empty(world * m, device=dev, dtype=dtype)
            comm.all_gather(g, shard)
            exp = torch.cat([torch.arange(m, device=dev, dtype=torch.float32).remainder(3) + 10 * r
                             for r in range(world)])
            res[f"ag_big_{dtype}"] = bool(torch.equal(g.float(), exp))
        # random non-integer data against an fp32 sum of every rank's (bf16-rounded) input: a rank
        # counted twice, a missing rank, a wrong scale or a shifted element all fail these (integer
        # patterns can hide a permutation)
        def rnd(r, n, dtype):
            g = torch.Generator(device=dev).manual_seed(1000 + 17 * r + n)
            return torch.randn(n, generator=g, device=dev).to(dtype)

        for dtype in (torch.float32, torch.bfloat16):
            for n in (3000, 100040, 3 * (1 << 20) // 4 + 4096):
                t = rnd(rank, n, dtype)
                comm.all_reduce(t)
                exp = sum(rnd(r, n, dtype).float() for r in range(world))
                tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
                res[f"ar_rand_{dtype}_{n}"] = bool(torch.allclose(t.float(), exp, rtol=tol, atol=tol))
                a = rnd(rank, n, dtype)
                comm.all_reduce(a, average=True)
                res[f"ar_rand_avg_{dtype}_{n}"] = bool(torch.allclose(a.float(), exp / world, rtol=tol, atol=tol))
            m = 40960
            x = rnd(rank, world * m, dtype)
            out = torch.empty(m, device=dev, dtype=dtype)
            comm.reduce_scatter(out, x)
            exp = sum(rnd(r, world * m, dtype).float() for r in range(world))[rank * m:(rank + 1) * m]
            tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
            res[f"rs_rand_{dtype}"] = bool(torch.allclose(out.float(), exp, rtol=tol, atol=tol))
        # many back-to-back calls: the slot parity / epoch protocol never desynchronises
        t = torch.ones(4096, device=dev)
        for _ in range(1000):
            comm.all_reduce(t, average=True)
        res["back_to_back"] = bool((t == 1.0).all().item())
        # slot wrap: two-shot calls alternating between the two slot parities with changing data
        u = torch.empty(world * 8192, device=dev)
        ok = True
        for k in range(20):
            u.fill_(float(k + rank))
            comm.all_reduce(u)
            ok &= bool((u == float(world * k + sum(range(world)))).all().item())
        res["slot_wrap"] = ok
        torch.cuda.synchronize()
        comm.check_error()
        # a peer that skips a collective: the waiting rank's barrier gives up and the NEXT check raises
        if skip:
            if rank == 0:
                comm.all_reduce(torch.ones(1024, device=dev))
                try:
                    comm.check_error()
                    res["skip_raises"] = False
                except XgmiError:
                    res["skip_raises"] = True
                comm.check_error()  # cleared after being reported once
            dist.barrier()
        comm.close()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, {"error": repr(e)}))
