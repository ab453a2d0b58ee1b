"""Rank body for tests/test_ps_plane_gpu.py: the dedicated PS over the xGMI data plane (csrc/ps_plane.hip),
every rank a process on the one GPU of the test box (gloo carries only the window-handle exchange)."""
import os

import torch
import torch.distributed as dist

import gpu_ranks


class _Net(torch.nn.Module):
    """Parameters only (the push / apply / land protocol does not care where gradients come from)."""

    def __init__(self, sizes):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(n)) for n in sizes])


def _grad_value(step, widx, i):
    """The gradient worker ``widx`` pushes at ``step`` for flat element ``i`` (exact in bf16)."""
    return float((widx + 1) * (step % 3 + 1)) * 0.25 + (i % 4) * 0.125


def _master_flat(ps):
    """The ps's fp32 masters (stored bucket by bucket) back in flat-buffer order."""
    master = ps.optimizers[ps.rank].w.cpu()
    out = torch.zeros(ps.flat.numel)
    for b in ps.buckets:
        m, n = ps._master_range[b.index]
        out[b.lo:b.hi] = master[m:m + n]
    return out


def run(rank, world, port, q, sync=True, wire=None, steps=4):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dev, _ = gpu_ranks.init(rank, world)
        from tony_amd.parallel.ps import ParameterServer

        torch.manual_seed(0)
        net = _Net([11000, 12000, 4136, 13000, 3000, 11008, 64])
        with torch.no_grad():
            for p in net.ps:
                p.copy_(torch.randn(p.shape).mul_(0.5))
        lr = 0.5
        ps = ParameterServer(net, optimizer="sgd", lr=lr, momentum=0.0, mode="dedicated", sync=sync,
                             ps_ranks=(0,), dtype=torch.bfloat16, device=dev, bucket_mb=0.02,
                             wire_dtype=wire, plane="xgmi")
        assert ps.plane is not None and len(ps.buckets) > 3
        n = ps.flat.numel
        w0 = ps.flat.data.float().cpu().clone()
        idx = torch.arange(n, dtype=torch.float32)
        nw = len(ps.worker_ranks)
        for s in range(steps):
            if ps.is_worker:
                ps.begin_step(overlap=False)
                widx = ps.worker_ranks.index(rank)
                g = float((widx + 1) * (s % 3 + 1)) * 0.25 + (idx.remainder(4)) * 0.125
                ps.flat.grad.copy_(g.to(dev))
            ps.step()
        torch.cuda.synchronize()
        ps.plane.check_error()
        res = {}
        # total pushed gradient per element, and this worker's own share
        tot = torch.zeros(n)
        own = torch.zeros(n)
        for s in range(steps):
            for w in range(nw):
                g = float((w + 1) * (s % 3 + 1)) * 0.25 + idx.remainder(4) * 0.125
                tot += g
                if ps.is_worker and w == ps.worker_ranks.index(rank):
                    own += g
        if sync:
            # sync, momentum 0: w = w0 - lr * sum_s mean_w g  (each step rounded to bf16 on the landing side,
            # the fp32 master carries the exact value)
            exp = w0 - lr * tot / nw
            got = ps.flat.data.float().cpu()
            res["params_match"] = bool(torch.allclose(got, exp, rtol=1e-2, atol=2e-2))
            if ps.is_ps:
                res["master_match"] = bool(torch.allclose(_master_flat(ps), exp, rtol=1e-5, atol=1e-4))
        else:
            # async, momentum 0: updates commute -> the ps ends at w0 - lr * (every push); a worker's last
            # landing includes all of its own pushes and a subset of the others'
            if ps.is_ps:
                res["master_match"] = bool(torch.allclose(_master_flat(ps), w0 - lr * tot, rtol=1e-5, atol=1e-3))
            else:
                applied = (w0 - ps.flat.data.float().cpu()) / lr
                res["own_included"] = bool((applied >= own * 0.99 - 0.1).all())
                res["bounded_by_total"] = bool((applied <= tot * 1.01 + 0.1).all())
        res["pushed"] = ps.plane.pushed
        ps.plane.close()
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback

        q.put((rank, {"error": f"{e!r}\n{traceback.format_exc()}"}))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_overlap(rank, world, port, q):
    """A small fused conv net trained through the Trainer on the xGMI plane: pushes launch during backward,
    every worker ends each step with the same parameters, and the run matches the RCCL-free reference
    order of a sync PS (loss finite, parameters changed)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dev, _ = gpu_ranks.init(rank, world)
        from tony_amd.models.layers import ConvBNAct, cast_model, init_weights
        from tony_amd.ops import cross_entropy
        from tony_amd.ops.pool import global_avg_pool
        from tony_amd.parallel.ps import ParameterServer
        from tony_amd.parallel.trainer import Trainer

        class Net(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.c1 = ConvBNAct(16, 64, 3, 1, 1)
                self.c2 = ConvBNAct(64, 64, 3, 1, 1)
                self.c3 = ConvBNAct(64, 128, 3, 2, 1)
                self.fc = torch.nn.Linear(128, 16)

            def forward(self, x):
                return self.fc(global_avg_pool(self.c3(self.c2(self.c1(x)))))

        model = cast_model(init_weights(Net(), seed=1), torch.bfloat16, dev).to(memory_format=torch.channels_last)
        ps = ParameterServer(model, optimizer="sgd", lr=0.05, momentum=0.9, mode="dedicated", ps_ranks=(0,),
                             dtype=torch.bfloat16, device=dev, bucket_mb=0.05, plane="xgmi")
        res = {}
        steps = 5
        import sys
        import time

        t0 = time.time()

        def say(msg):
            print(f"[rank {rank} t={time.time() - t0:.1f}s] {msg}", file=sys.stderr, flush=True)

        if ps.is_ps:
            for s_ in range(steps):
                ps.step()
                say(f"ps step {s_} issued")
        else:
            trainer = Trainer(model, ps, lambda out, y: cross_entropy(out, y), use_graph=False)
            g = torch.Generator(device=dev).manual_seed(rank)
            x = torch.randn((16, 16, 24, 24), generator=g, device=dev).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            y = torch.randint(0, 16, (16,), generator=g, device=dev)
            overl = []
            if os.environ.get("TONY_PS_PLANE_TRACE"):
                # progress of the first step, phase by phase (diagnostics for a stalled rehearsal)
                orig_step, orig_bwd = ps.step, torch.Tensor.backward

                def traced_step():
                    say("ps.step (pushes + land) issuing")
                    orig_step()
                    say("ps.step issued")

                def traced_bwd(t, *a, **k):
                    say("backward start")
                    orig_bwd(t, *a, **k)
                    say("backward issued")

                ps.step = traced_step
                torch.Tensor.backward = traced_bwd
            for s_ in range(steps):
                say(f"worker step {s_} start")
                loss = trainer.step(x, y)
                torch.cuda.synchronize()
                say(f"worker step {s_} done (overlapped buckets {ps.overlapped_buckets} of {len(ps.buckets)})")
                overl.append(ps.overlapped_buckets)
            res["loss_finite"] = bool(torch.isfinite(loss).item())
            res["overlapped"] = max(overl) > 0
        torch.cuda.synchronize()
        ps.plane.check_error()
        flat = ps.flat.data.float().cpu()
        allf = [None] * world
        dist.all_gather_object(allf, flat)
        res["workers_agree"] = all(torch.equal(allf[w], allf[ps.worker_ranks[0]]) for w in ps.worker_ranks)
        res["ps_matches_workers"] = bool(torch.equal(allf[0], allf[ps.worker_ranks[0]]))
        ps.plane.close()
        if ps.is_ps:
            # reference: the same sync-PS trajectory in one process -- each step every worker's gradient
            # on its own batch (same fused kernels), their mean, SGD-momentum on an fp32 master, the
            # bf16 copy for the next step.  Agreement among the ranks alone would pass a wrong-but-
            # consistent sum (a worker dropped or counted twice, a missing 1/n).
            ref = cast_model(init_weights(Net(), seed=1), torch.bfloat16, dev).to(memory_format=torch.channels_last)
            names = [n for n, _ in ref.named_parameters()]
            master = {n: p.detach().float().clone() for n, p in ref.named_parameters()}
            w0 = {n: t.clone() for n, t in master.items()}
            mom = {n: torch.zeros_like(t) for n, t in master.items()}
            batches = []
            for w in ps.worker_ranks:
                gw = torch.Generator(device=dev).manual_seed(w)
                xw = torch.randn((16, 16, 24, 24), generator=gw, device=dev).to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
                batches.append((xw, torch.randint(0, 16, (16,), generator=gw, device=dev)))
            for _ in range(steps):
                gsum = {n: torch.zeros_like(t) for n, t in master.items()}
                for xw, yw in batches:
                    for p in ref.parameters():
                        p.grad = None
                    cross_entropy(ref(xw), yw).backward()
                    for n, p in ref.named_parameters():
                        gsum[n] += p.grad.float()
                with torch.no_grad():
                    for n, p in ref.named_parameters():
                        mom[n].mul_(0.9).add_(gsum[n] / len(batches))
                        master[n].sub_(0.05 * mom[n])
                        p.copy_(master[n].to(p.dtype))
            got = dict(model.named_parameters())
            num = sum(float((got[n].float() - w0[n] - (master[n] - w0[n])).norm() ** 2) for n in names) ** 0.5
            den = sum(float((master[n] - w0[n]).norm() ** 2) for n in names) ** 0.5
            res["update_rel_err_vs_reference"] = num / max(den, 1e-12)
            res["matches_reference"] = res["update_rel_err_vs_reference"] < 0.05
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, {"error": f"{e!r}\n{traceback.format_exc()}"}))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
