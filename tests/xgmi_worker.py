"""Rank body for tests/test_xgmi_gpu.py (importable by spawned processes)."""
import os

import torch
import torch.distributed as dist


def run(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)  # every rank on the one GPU of the test box: IPC + the protocol
        from tony_amd.parallel.xgmi import XgmiComm

        comm = XgmiComm(slot_bytes=1 << 20, oneshot_max_bytes=64 << 10, blocks=8)
        dev = torch.device("cuda", 0)
        res = {}
        for dtype in (torch.float32, torch.bfloat16):
            for n in (1024, 40960, 3 * (1 << 20) // 4 + 4096):  # one-shot, two-shot, multi-piece
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
        torch.cuda.synchronize()
        comm.check_error()
        comm.close()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, {"error": repr(e)}))
