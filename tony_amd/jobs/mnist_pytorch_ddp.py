"""MNIST with synchronous data parallelism under TonY's pytorch runtime
(the job of EX/mnist-pytorch/mnist_distributed.py, README: framework=pytorch, ps=0, workers=2).

The reference averages each parameter's gradient with its own CPU all_reduce and a new group per
call; here the model is wrapped in tony_amd's bucketed DDP (one flat gradient buffer, RCCL
all-reduce over xGMI on GPUs, gloo on CPU) and the process group comes from the pytorch runtime's
env contract (INIT_METHOD / RANK / WORLD plus MASTER_ADDR / MASTER_PORT / WORLD_SIZE / LOCAL_RANK).
Data is a deterministic synthetic MNIST-shaped set sharded by rank (DistributedSampler semantics).

usage (through TonY):
  tony --src_dir tony_amd/jobs --executes mnist_pytorch_ddp.py \
       --conf tony.application.framework=pytorch --conf tony.worker.instances=2 [--task_params "--epochs 2"]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from tony_amd.jobs.common import Throughput, log, metric, working_dir  # noqa: E402
from tony_amd.models.mnist import mnist_model, synthetic_mnist  # noqa: E402
from tony_amd.parallel import bootstrap  # noqa: E402
from tony_amd.parallel.ddp import DistributedDataParallel  # noqa: E402
from tony_amd.utils.checkpoint import CheckpointManager, resume_step, training_state  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="linear", choices=["linear", "deepnn", "keras_cnn", "hvd_cnn", "dnn"])
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--steps-per-epoch", type=int, default=20)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.5)
    ap.add_argument("--checkpoint-steps", type=int, default=0)
    a = ap.parse_args(argv)
    rank, world, _, dev = bootstrap.init_from_env()
    log(f"rank {rank}/{world} on {dev}")
    model = mnist_model(a.model, seed=0).to(dev)
    ddp = DistributedDataParallel(model)
    opt = torch.optim.SGD(model.parameters(), lr=a.lr, momentum=a.momentum)
    ckpt = CheckpointManager(os.path.join(working_dir(), "mnist_ddp"), save_steps=a.checkpoint_steps, rank=rank)
    state = ckpt.restore(map_location=dev) if a.checkpoint_steps else None
    step = resume_step(state)
    if state:
        model.load_state_dict(state["model"])
        opt.load_state_dict(state["optimizer"])
        log(f"resumed from step {step}")
    x_all, y_all = synthetic_mnist(a.batch_size * world * a.steps_per_epoch, seed=1, device=dev)
    tp = Throughput(dev)
    first = last = None
    for epoch in range(a.epochs):
        tp.start()
        for i in range(a.steps_per_epoch):
            lo = (i * world + rank) * a.batch_size  # this rank's shard of the global batch
            x, y = x_all[lo:lo + a.batch_size], y_all[lo:lo + a.batch_size]
            ddp.zero_grad()
            loss = torch.nn.functional.cross_entropy(ddp(x), y)
            loss.backward()
            opt.step()
            step += 1
            tp.add(x.shape[0])
            last = float(loss)
            first = last if first is None else first
            ckpt.save(step, training_state(model, opt))
        metric(epoch=epoch, loss=last, samples_per_sec=tp.rate() * world, rank=rank)
    ckpt.wait()
    log(f"loss {first:.4f} -> {last:.4f}")
    torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
