"""Horovod MNIST under TonY's horovod runtime
(the job of EX/horovod-on-tony/tensorflow2_mnist.py: pin the GPU by local rank, scale the Adam
learning rate by size, DistributedGradientTape-style gradient averaging, broadcast the initial
variables and optimizer state from rank 0, rank-0 checkpoint).

The ``hvd`` module is tony_amd's Horovod-compatible API: ranks come from the HOROVOD_* env the
runtime injects and the torch process group rendezvouses through the driver's HTTP KV store.

  tony --src_dir tony_amd/jobs --executes hvd_mnist.py --conf tony.application.framework=horovod \
       --conf tony.worker.instances=2
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import tony_amd.hvd as hvd  # noqa: E402
from tony_amd.jobs.common import log, metric, working_dir  # noqa: E402
from tony_amd.models.mnist import mnist_model, synthetic_mnist  # noqa: E402
from tony_amd.utils.checkpoint import CheckpointManager  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--lr", type=float, default=0.001)
    a = ap.parse_args(argv)
    hvd.init()
    dev = hvd.device()
    log(f"hvd rank {hvd.rank()}/{hvd.size()} local {hvd.local_rank()}/{hvd.local_size()} on {dev}")
    model = mnist_model("hvd_cnn", seed=hvd.rank()).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=a.lr * hvd.size())
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters())
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    x_all, y_all = synthetic_mnist(a.batch_size * hvd.size() * 4, seed=7, device=dev)
    losses = []
    for s in range(a.steps):
        lo = ((s % 4) * hvd.size() + hvd.rank()) * a.batch_size
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x_all[lo:lo + a.batch_size]), y_all[lo:lo + a.batch_size])
        loss.backward()
        opt.step()
        losses.append(float(loss))
    avg_last = float(hvd.allreduce(torch.tensor([losses[-1]])))  # MetricAverageCallback
    if hvd.rank() == 0:
        ckpt = CheckpointManager(os.path.join(working_dir(), "hvd_mnist"), rank=0)
        ckpt.save(a.steps, {"model": model.state_dict()}, force=True)
        ckpt.wait()
        metric(first_loss=losses[0], avg_last_loss=avg_last, size=hvd.size())
    log(f"loss {losses[0]:.4f} -> {losses[-1]:.4f} (avg over ranks {avg_last:.4f})")
    hvd.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
