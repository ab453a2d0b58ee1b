"""MNIST with synchronous all-reduce driven by TF_CONFIG
(the job of EX/mnist-tensorflow/mnist_keras_distributed.py: MultiWorkerMirroredStrategy over the
TF_CONFIG workers, global batch = 64 x number of workers, SGD(momentum=0.5), the Keras CNN).

MultiWorkerMirroredStrategy all-reduces gradients every step; here that is tony_amd's bucketed
DDP over the process group TF_CONFIG describes (chief/worker ranks; RCCL on GPUs, gloo on CPU).

  tony --src_dir tony_amd/jobs --executes mnist_tf_allreduce.py --conf tony.worker.instances=3 \
       --conf tony.ps.instances=0
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from tony_amd.jobs.common import log, metric  # noqa: E402
from tony_amd.models.mnist import mnist_model, synthetic_mnist  # noqa: E402
from tony_amd.parallel import bootstrap  # noqa: E402
from tony_amd.parallel.ddp import DistributedDataParallel  # noqa: E402
from tony_amd.parallel.tf_config import TFConfig  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-worker-batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lr", type=float, default=0.001)
    a = ap.parse_args(argv)
    tc = TFConfig.from_env().without_ps()
    rank, world, dev = bootstrap.init_from_tf_config(tc)
    global_batch = tc.global_batch(a.per_worker_batch)
    model = mnist_model("keras_cnn", seed=0).to(dev)
    ddp = DistributedDataParallel(model)
    opt = torch.optim.SGD(model.parameters(), lr=a.lr, momentum=0.5)
    x_all, y_all = synthetic_mnist(global_batch * 4, seed=3, device=dev)
    losses = []
    for s in range(a.steps):
        lo = (s % 4) * global_batch + rank * a.per_worker_batch
        ddp.zero_grad()
        loss = torch.nn.functional.cross_entropy(ddp(x_all[lo:lo + a.per_worker_batch]),
                                                 y_all[lo:lo + a.per_worker_batch])
        loss.backward()
        opt.step()
        losses.append(float(loss))
    metric(global_batch=global_batch, first_loss=losses[0], last_loss=losses[-1], rank=rank)
    log(f"{tc.task_type}:{tc.task_index} global batch {global_batch}: loss {losses[0]:.4f} -> {losses[-1]:.4f}")
    torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
