"""Linear regression through the MXNet-style kvstore under TonY's mxnet runtime
(the job of EX/linearregression-mxnet/src/mxnet_dist_ex.py: 75,000 training rows of y = f(x),
batch 1024, one FullyConnected(num_hidden=1) layer, ``kvstore='dist_async'``; BASELINE.json
names the ``dist_sync`` 1 ps + 8 workers config).

Roles follow DMLC_ROLE: the ``scheduler`` task hosts the rendezvous store, ``server`` tasks own
the weights and run the optimizer, ``worker`` tasks compute gradients on their shard of the data
and push / pull through ``tony_amd.kv`` (``import mxnet`` runs the non-worker roles implicitly;
here ``kv.run_role()`` does).

  tony --src_dir tony_amd/jobs --executes mxnet_linreg.py --conf tony.application.framework=mxnet \
       --conf tony.scheduler.instances=1 --conf tony.server.instances=1 --conf tony.worker.instances=2 \
       [--task_params "--kvstore dist_sync"]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import tony_amd.kv as kv  # noqa: E402
from tony_amd.jobs.common import log, metric  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kvstore", default="dist_async")
    ap.add_argument("--rows", type=int, default=75000)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--lr", type=float, default=0.1)
    a = ap.parse_args(argv)
    if kv.run_role():  # scheduler / server: serve until the workers are done
        return 0
    store = kv.create(a.kvstore)
    rank, nw = store.rank, store.num_workers
    g = torch.Generator().manual_seed(0)
    x = torch.rand(a.rows, 1, generator=g) * 2 - 1
    y = 3.0 * x[:, 0] + 0.5 + 0.01 * torch.randn(a.rows, generator=g)
    shard = slice(rank * a.rows // nw, (rank + 1) * a.rows // nw)  # this worker's part of the data
    xs, ys = x[shard], y[shard]
    w, b = torch.zeros(1, 1), torch.zeros(1)
    store.init("fc_weight", w)
    store.init("fc_bias", b)
    store.set_optimizer(kv.create_optimizer("sgd", learning_rate=a.lr, rescale_grad=1.0 / (a.batch_size * nw)))
    mse = None
    for epoch in range(a.epochs):
        for lo in range(0, xs.shape[0], a.batch_size):
            xb, yb = xs[lo:lo + a.batch_size], ys[lo:lo + a.batch_size]
            err = (xb @ w.t())[:, 0] + b - yb                       # forward of FullyConnected(1)
            store.push("fc_weight", 2 * (err[:, None] * xb).sum(0, keepdim=True))   # d(sum err^2)/dw
            store.push("fc_bias", 2 * err.sum(0, keepdim=True))
            store.pull("fc_weight", out=w)
            store.pull("fc_bias", out=b)
        mse = float((((x @ w.t())[:, 0] + b - y) ** 2).mean())
        metric(epoch=epoch, mse=mse, rank=rank)
    log(f"worker {rank}/{nw}: w={float(w):.3f} b={float(b):.3f} mse={mse:.5f}")
    store.close()
    return 0 if mse < 0.05 else 1


if __name__ == "__main__":
    sys.exit(main())
