"""ResNet-50 bf16 data-parallel training through the PyTorch runtime (SURVEY.md §7.3's minimum slice:
ClusterSubmitter -> coordinator -> N task agents pinned to GPUs -> PyTorch env contract
(INIT_METHOD / RANK / WORLD + MASTER_ADDR / MASTER_PORT / LOCAL_RANK / WORLD_SIZE) ->
init_process_group("nccl") = RCCL over xGMI).

Per rank: the fused-kernel ResNet-50 (NHWC bf16, tony_amd BN / GEMM / residual / conv HIP kernels),
synthetic ImageNet batches generated on the device, tony_amd's DistributedDataParallel (gradients
in one flat buffer, bucketed all-reduce launched from the backward hooks, so communication overlaps
the rest of the backward), SGD-momentum.  Reports images/sec over all ranks.

  tony --src_dir tony_amd/jobs --executes resnet50_ddp.py --conf tony.application.framework=pytorch \
       --conf tony.worker.instances=8 --conf tony.worker.gpus=1 --conf tony.ps.instances=0 \
       --conf tony.worker.memory=32g
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from tony_amd.jobs.common import Throughput, log, metric, synthetic_images  # noqa: E402
from tony_amd.models.layers import cast_model  # noqa: E402
from tony_amd.models.resnet import resnet50  # noqa: E402
from tony_amd.parallel import bootstrap  # noqa: E402
from tony_amd.parallel import collectives as coll  # noqa: E402
from tony_amd.parallel.ddp import DistributedDataParallel  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=32)
    a = ap.parse_args(argv)
    rank, world, _, dev = bootstrap.init_from_env()
    on_gpu = dev.type == "cuda"
    dtype = torch.bfloat16 if on_gpu else torch.float32
    if on_gpu:
        torch.backends.cudnn.benchmark = True
    model = cast_model(resnet50(fused=on_gpu), dtype, dev).to(memory_format=torch.channels_last)
    ddp = DistributedDataParallel(model, bucket_mb=a.bucket_mb)
    opt = torch.optim.SGD(model.parameters(), lr=0.1 * world, momentum=0.9, weight_decay=5e-5)
    x, y = synthetic_images(a.batch_size, a.image_size, 1000, dev, dtype, seed=rank)
    tp = Throughput(dev)
    loss = None
    for s in range(a.warmup + a.steps):
        if s == a.warmup:
            if world > 1:
                torch.distributed.barrier()
            tp.start()
        ddp.zero_grad()
        loss = torch.nn.functional.cross_entropy(ddp(x).float(), y)
        loss.backward()
        opt.step()
        if s >= a.warmup:
            tp.add(a.batch_size)
    rate = tp.rate()
    if world > 1:
        t = torch.tensor([rate], dtype=torch.float64, device=dev)
        coll.all_reduce(t)
        rate = float(t.item())
    if rank == 0:
        metric(model="resnet50", images_per_sec=rate, world=world, batch_per_rank=a.batch_size, loss=float(loss))
    log(f"{rate:.1f} images/sec over {world} ranks")
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
