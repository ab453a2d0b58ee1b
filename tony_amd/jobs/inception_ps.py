"""Inception-v3 parameter-server training driven by TF_CONFIG -- the headline job
(BASELINE.json: "Inception-v3 TF ParameterServerStrategy 1 ps + 4 workers on 4xMI355X").

PS semantics without TensorFlow (SURVEY.md §7.4 hard part 1): the ps tasks of TF_CONFIG own the
variables and apply the optimizer, workers push gradients and pull variables every step.

``--ps-mode colocated`` (default when the ps tasks have no GPU of their own)
    Each worker GPU hosts one shard of the variables: push = RCCL reduce-scatter over xGMI, apply
    = the fused HIP SGD on the shard's fp32 master copy, pull = all-gather.  The ``ps`` tasks of
    the cluster spec do what a TF ps does once the graph is placed -- ``server.join()`` -- and are
    stopped by the coordinator when training ends (ps is untracked by default).
``--ps-mode dedicated``
    The ps task(s) join the group and own the variables (give them GPUs: tony.ps.gpus=1).

The step (forward, loss, backward, push/apply/pull) is captured once into a HIP graph.

  tony --src_dir tony_amd/jobs --executes inception_ps.py --conf tony.ps.instances=1 \
       --conf tony.worker.instances=4 --conf tony.worker.gpus=1
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tony_amd.jobs.common import Throughput, log, metric, synthetic_images  # noqa: E402
from tony_amd.parallel import bootstrap  # noqa: E402
from tony_amd.parallel.ps import ParameterServer  # noqa: E402
from tony_amd.parallel.tf_config import TFConfig  # noqa: E402
from tony_amd.parallel.trainer import Trainer  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ps-mode", default="auto", choices=["auto", "colocated", "dedicated"])
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--image-size", type=int, default=299)
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args(argv)
    tc = TFConfig.from_env()
    on_gpu = torch.cuda.is_available()
    mode = a.ps_mode
    if mode == "auto":  # every task must decide the same way: only from the shared conf / env
        mode = os.environ.get("TONY_PS_MODE", "colocated" if on_gpu else "dedicated")
    if mode == "colocated":
        if tc.task_type == "ps":
            log("colocated PS: variables are sharded over the worker GPUs; ps task joins (waits) until stopped")
            while True:
                time.sleep(3600)
        tc = tc.without_ps()
    rank, world, dev = bootstrap.init_from_tf_config(tc)
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.models.layers import cast_model

    dtype = torch.bfloat16 if on_gpu else torch.float32
    if on_gpu:
        torch.backends.cudnn.benchmark = True
    model = cast_model(inception_v3(fused=on_gpu, seed=0), dtype, dev).to(memory_format=torch.channels_last)
    ps = ParameterServer(model, optimizer="sgd", lr=0.045, momentum=0.9, weight_decay=4e-5, mode=mode,
                         ps_ranks=tc.ps_ranks if mode == "dedicated" else (0,), dtype=dtype, device=dev)
    if mode == "dedicated" and ps.is_ps and not ps.is_worker:
        for _ in range(a.warmup + a.steps):
            ps.step()
        dist.barrier()
        return 0

    def loss_fn(out, y):
        logits, aux = out if isinstance(out, tuple) else (out, None)
        loss = torch.nn.functional.cross_entropy(logits.float(), y)
        if aux is not None:
            loss = loss + 0.4 * torch.nn.functional.cross_entropy(aux.float(), y)
        return loss

    trainer = Trainer(model, ps, loss_fn, use_graph=on_gpu and not a.no_graph)
    x, y = synthetic_images(a.batch_size, a.image_size, 1000, dev, dtype, seed=rank)
    tp = Throughput(dev)
    for s in range(a.warmup + a.steps):
        if s == a.warmup:
            dist.barrier()
            tp.start()
        loss = trainer.step(x, y)
        if s >= a.warmup:
            tp.add(a.batch_size)
    rate = torch.tensor([tp.rate()], dtype=torch.float64, device=dev if on_gpu else "cpu")
    dist.all_reduce(rate)
    workers = len(ps.worker_ranks)
    if tc.is_chief or rank == 0:
        metric(model="inception_v3", images_per_sec=float(rate), workers=workers, ps_mode=mode, loss=float(loss))
    log(f"{float(rate):.1f} images/sec total over {workers} workers ({mode} PS)")
    dist.barrier()
    return 0


if __name__ == "__main__":
    sys.exit(main())
