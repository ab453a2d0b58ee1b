"""Rank body of tests/test_x3_ps_gpu.py: the x3 (fp32) Inception-v3 trained through the ParameterServer
(colocated or dedicated) by N processes, then checked against a single-process reference of the same sync-PS
step (per-worker forward / backward on that worker's batch, gradients averaged, SGD-momentum with L2 decay
in fp32 -- optim_math.h sgd_update4's formula)."""
import os

import torch

import gpu_ranks

B, STEPS, CLASSES = 2, 2, 1000  # (the x3 classifier wants out_features % 8 == 0)
LR, MU, WD = 0.1, 0.9, 4e-5


def _data(w, dev):
    g = torch.Generator(device=dev).manual_seed(77 + w)
    x = torch.randn((B, 3, 299, 299), generator=g, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, CLASSES, (B,), generator=g, device=dev)
    return x, y


def _model(dev):
    from tony_amd.models.inception_v3 import inception_v3

    torch.manual_seed(0)
    m = inception_v3(num_classes=CLASSES, precision="fp32", seed=0).to(dev).to(memory_format=torch.channels_last)
    m.dropout.p = 0.0  # the reference replays the workers' forwards: no masks to match
    return m.train()


def _loss(out, y):
    from tony_amd.ops import cross_entropy

    logits, aux = out
    return cross_entropy(logits, y) + 0.4 * cross_entropy(aux, y)


def _say(rank, msg):
    import sys
    import time

    print(f"[x3-ps rank {rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def run(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if os.environ.get("X3PS_DUMP_S"):  # diagnostics: every rank's Python stack after that many seconds
        import faulthandler
        import sys

        faulthandler.dump_traceback_later(int(os.environ["X3PS_DUMP_S"]), repeat=False, file=sys.stderr)
    res = {}
    try:
        dev, _ = gpu_ranks.init(rank, world)
        import torch.distributed as dist

        from tony_amd.parallel.ps import ParameterServer
        from tony_amd.parallel.trainer import Trainer

        first = 0 if mode == "colocated" else 1
        nw = world if mode == "colocated" else world - 1
        if rank == first:
            # single-process reference first (no parameter server attached in this process yet): same init,
            # each worker's batch through a fresh x3 model, mean gradient, fp32 SGD-momentum + L2 -- run
            # TWICE: the two runs differ by the network's own sensitivity (the order of the fp32 atomics in
            # the BN statistics moves y by ~1e-7, a ReLU mask bit flips wherever |y| is that small, and 95 BN
            # layers at batch 2 amplify each flip -- tools/x3_layer_check.py shows one layer's flips at the
            # x3 forward precision), which is the yardstick for the PS run
            trajs = []
            for _ in range(2):
                ref = _model(dev)
                params = list(ref.parameters())
                w0 = [p.detach().clone() for p in params]
                vel = [torch.zeros_like(p) for p in params]
                drs = []
                for _ in range(STEPS):
                    gsum = [torch.zeros_like(p) for p in params]
                    for w in range(nw):
                        for p in params:
                            p.grad = None
                        xw, yw = _data(w, dev)
                        _loss(ref(xw), yw).backward()
                        _say(rank, f"reference: worker {w}'s batch done")
                        for s_, p in zip(gsum, params):
                            s_ += p.grad
                    with torch.no_grad():
                        for p, v, s_ in zip(params, vel, gsum):
                            v.mul_(MU).add_(s_ / nw + WD * p)
                            p.add_(v, alpha=-LR)
                    drs.append(torch.cat([(a.detach() - b).flatten() for a, b in zip(params, w0)]))
                trajs.append(drs)
                del ref, params, vel, gsum
            drs = trajs[0]
            dr = drs[-1]
            res["ref_spread_per_step"] = [float((u - r).norm() / r.norm()) for u, r in zip(trajs[1], drs)]
            del trajs
            torch.cuda.synchronize()
        dist.barrier()  # every rank starts the parameter server together (the reference took minutes)
        model = _model(dev)
        ps = ParameterServer(model, optimizer="sgd", lr=LR, momentum=MU, weight_decay=WD, mode=mode, ps_ranks=(0,),
                             dtype=torch.float32, device=dev, wire_dtype=torch.float32,
                             bucket_mb=float(os.environ.get("X3PS_BUCKET_MB", "8")))
        workers = list(ps.worker_ranks)
        assert workers[0] == first and len(workers) == nw, (workers, first, nw)
        if ps.is_worker:
            # (diagnostic switches for the dedicated rehearsal: X3PS_OVERLAP=0 pushes after backward,
            # X3PS_BRANCH=0 keeps the blocks' branches on one stream)
            trainer = Trainer(model, ps, _loss, use_graph=False,
                              overlap_comm=os.environ.get("X3PS_OVERLAP", "1") != "0",
                              branch_streams=os.environ.get("X3PS_BRANCH", "1") != "0")
            x, y = _data(workers.index(rank), dev)
            dus = []
            for i in range(STEPS):
                loss = trainer.step(x, y)
                torch.cuda.synchronize()
                _say(rank, f"PS step {i} done")
                if rank == first:
                    dus.append(torch.cat([(p.detach() - b).flatten() for p, b in zip(model.parameters(), w0)]))
            res["loss_finite"] = bool(torch.isfinite(loss).item())
        else:
            for i in range(STEPS):
                ps.step()
                _say(rank, f"ps apply {i} issued")
            torch.cuda.synchronize()
        dist.barrier()
        if rank == first:
            du = torch.cat([(p.detach() - b).flatten() for p, b in zip(model.parameters(), w0)])
            res["update_rel_err"] = float((du - dr).norm() / dr.norm())
            res["update_rel_err_per_step"] = [float((u - r).norm() / r.norm()) for u, r in zip(dus, drs)]
            # which parameters disagree most after the first step (diagnosis)
            worst, off = [], 0
            for (name, p_), b in zip(model.named_parameters(), w0):
                k = p_.numel()
                u, r = dus[0][off:off + k], drs[0][off:off + k]
                worst.append((float((u - r).norm() / (r.norm() + 1e-30)), name, k))
                off += k
            res["worst_params_step0"] = sorted(worst, reverse=True)[:6]
            _say(rank, f"result: {res}")
            res["update_norm"] = float(dr.norm())
            res["plane"] = getattr(ps, "plane_kind", None)
            res["workers"] = len(workers)
        if ps.plane is not None:
            ps.plane.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - reported to the test
        import traceback

        res["error"] = f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2500:]}"
    q.put((rank, res))
