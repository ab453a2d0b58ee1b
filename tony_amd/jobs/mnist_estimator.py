"""MNIST "Estimator" job: chief / worker / ps / evaluator roles from TF_CONFIG
(the job of EX/mnist-tensorflow/mnist_estimator_distributed.py: ``train_and_evaluate`` with a
DNNClassifier([256, 128]), ``RunConfig(save_checkpoints_steps, keep_checkpoint_max=3)``).

* chief + workers train through a dedicated synchronous ParameterServer on the ps task(s);
* the chief checkpoints every ``--save-steps`` steps into the model dir (keep 3) and writes a
  ``DONE`` marker at the end;
* the evaluator is not in the training group (its TF_CONFIG cluster has no other evaluator and
  TonY drops it from everyone else's view): it polls the model dir, evaluates each new
  checkpoint on held-out synthetic data, and exits after evaluating the final one.

Adagrad (the Estimator default) is replaced by the fused Adam of tony_amd.ops.optim.

  tony --src_dir tony_amd/jobs --executes mnist_estimator.py --conf tony.chief.instances=1 \
       --conf tony.worker.instances=2 --conf tony.ps.instances=1 --conf tony.evaluator.instances=1
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tony_amd.jobs.common import log, metric, working_dir  # noqa: E402
from tony_amd.models.mnist import mnist_model, synthetic_mnist  # noqa: E402
from tony_amd.parallel import bootstrap  # noqa: E402
from tony_amd.parallel.flat import FlatParams  # noqa: E402
from tony_amd.parallel.ps import ParameterServer  # noqa: E402
from tony_amd.parallel.tf_config import TFConfig  # noqa: E402
from tony_amd.utils.checkpoint import CheckpointManager  # noqa: E402


def evaluate(a, model_dir: str) -> int:
    model = mnist_model("dnn", seed=0)
    flat = FlatParams(model, dtype=torch.float32)
    ckpt = CheckpointManager(model_dir, rank=1)  # read-only view
    x, y = synthetic_mnist(512, seed=99)
    seen = set()
    deadline = time.time() + a.eval_timeout
    while time.time() < deadline:
        for step, path in ckpt.checkpoints():
            if step in seen:
                continue
            try:
                st = torch.load(path, weights_only=True)
            except (OSError, RuntimeError):
                continue  # being rotated out by keep_checkpoint_max
            seen.add(step)
            flat.data.copy_(st["flat"])
            with torch.no_grad():
                acc = (model(x).argmax(1) == y).float().mean().item()
            metric(eval_step=step, accuracy=acc)
            log(f"evaluated checkpoint {step}: accuracy {acc:.3f}")
        if os.path.exists(os.path.join(model_dir, "DONE")) and (not ckpt.checkpoints()
                                                                or ckpt.latest()[0] in seen):
            return 0
        time.sleep(0.2)
    log("evaluator timed out waiting for the final checkpoint")
    return 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--save-steps", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--eval-timeout", type=float, default=600)
    a = ap.parse_args(argv)
    tc = TFConfig.from_env()
    model_dir = working_dir("estimator_model")
    if tc.is_evaluator:
        return evaluate(a, model_dir)
    rank, world, dev = bootstrap.init_from_tf_config(tc)
    model = mnist_model("dnn", seed=0).to(dev)
    ps = ParameterServer(model, optimizer="adam", lr=1e-3, mode="dedicated", sync=True, ps_ranks=tc.ps_ranks,
                         dtype=torch.float32, device=dev)
    ckpt = CheckpointManager(model_dir, keep_max=3, save_steps=a.save_steps, rank=0 if tc.is_chief else 1)
    if tc.is_chief and os.path.exists(os.path.join(model_dir, "DONE")):
        os.remove(os.path.join(model_dir, "DONE"))
    x_all, y_all = synthetic_mnist(a.batch_size * max(1, len(ps.worker_ranks)) * 4, seed=5, device=dev)
    widx = ps.worker_ranks.index(rank) if ps.is_worker else -1
    for s in range(1, a.steps + 1):
        if ps.is_worker:
            lo = (((s - 1) % 4) * len(ps.worker_ranks) + widx) * a.batch_size
            ps.zero_grad()
            torch.nn.functional.cross_entropy(model(x_all[lo:lo + a.batch_size]),
                                              y_all[lo:lo + a.batch_size]).backward()
        ps.step()
        ckpt.save(s, {"flat": ps.flat.data})
    if tc.is_chief:
        ckpt.save(a.steps, {"flat": ps.flat.data}, force=not ckpt.should_save(a.steps))
        ckpt.wait()
        open(os.path.join(model_dir, "DONE"), "w").close()
        log(f"chief finished {a.steps} steps; checkpoints {[s for s, _ in ckpt.checkpoints()]}")
    dist.barrier()
    return 0


if __name__ == "__main__":
    sys.exit(main())
