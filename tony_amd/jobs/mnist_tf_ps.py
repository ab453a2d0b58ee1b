"""MNIST between-graph parameter-server training under TonY's tensorflow runtime
(the job of EX/mnist-tensorflow/mnist_distributed.py: ``ps`` tasks hold the variables of the
``deepnn`` model and apply Adam, workers pull variables / push gradients; asynchronous by default,
as TF's between-graph replication is).

Cluster membership comes from TF_CONFIG (or the low-level CLUSTER_SPEC + JOB_NAME + TASK_INDEX
contract the reference script reads).  The PS is tony_amd's ParameterServer in ``dedicated``
mode: the ps rank owns the fp32 master copy and optimizer state and runs the fused optimizer on
every push.  Worker 0 is the chief: it checkpoints (MonitoredTrainingSession's
``checkpoint_dir``) and, like the reference, owns TensorBoard's ``TB_PORT`` when TonY reserved
one (it records the port it would serve on).

  tony --src_dir tony_amd/jobs --executes mnist_tf_ps.py \
       --conf tony.ps.instances=1 --conf tony.worker.instances=2 [--task_params "--steps 200 --sync"]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tony_amd.jobs.common import log, metric, working_dir  # noqa: E402
from tony_amd.models.mnist import mnist_model, synthetic_mnist  # noqa: E402
from tony_amd.parallel import bootstrap  # noqa: E402
from tony_amd.parallel.ps import ParameterServer  # noqa: E402
from tony_amd.parallel.tf_config import TFConfig  # noqa: E402
from tony_amd.utils.checkpoint import CheckpointManager  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--sync", action="store_true", help="SyncReplicas semantics instead of async")
    ap.add_argument("--model", default="deepnn")
    a = ap.parse_args(argv)
    tc = TFConfig.from_env()
    if not tc.ps_ranks:
        log("no ps tasks in the cluster spec")
        return 1
    rank, world, dev = bootstrap.init_from_tf_config(tc)
    model = mnist_model(a.model, seed=0).to(dev)
    ps = ParameterServer(model, optimizer="adam", lr=a.lr, mode="dedicated", sync=a.sync, ps_ranks=tc.ps_ranks,
                         dtype=torch.float32, device=dev)
    if ps.is_ps:
        log(f"ps rank {rank}: serving {ps.flat.numel} variables ({'sync' if a.sync else 'async'})")
        if not a.sync:
            ps.serve_async(total_pushes=a.steps * len(ps.worker_ranks))
        else:
            for _ in range(a.steps):
                ps.step()
        dist.barrier()
        return 0
    if tc.is_chief and os.environ.get("TB_PORT"):
        log(f"chief owns TensorBoard port {os.environ['TB_PORT']}")
    widx = ps.worker_ranks.index(rank)
    x_all, y_all = synthetic_mnist(a.batch_size * len(ps.worker_ranks) * 4, seed=2, device=dev)
    losses = []
    for s in range(a.steps):
        lo = ((s % 4) * len(ps.worker_ranks) + widx) * a.batch_size
        ps.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x_all[lo:lo + a.batch_size]), y_all[lo:lo + a.batch_size])
        loss.backward()
        ps.step()
        losses.append(float(loss))
    if tc.is_chief:
        ckpt = CheckpointManager(os.path.join(working_dir(), "mnist_ps"), rank=0)
        ckpt.save(a.steps, {"flat": ps.flat.data}, force=True)
        ckpt.wait()
    metric(first_loss=losses[0], last_loss=losses[-1], worker=widx)
    log(f"worker {widx}: loss {losses[0]:.4f} -> {losses[-1]:.4f}")
    dist.barrier()
    return 0


if __name__ == "__main__":
    sys.exit(main())
