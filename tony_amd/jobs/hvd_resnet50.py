"""ResNet-50 bf16 data-parallel training through the Horovod API (BASELINE.json config
"horovod-on-tony ResNet-50 ring-allreduce bf16 on 8xMI355X").

Per rank: the fused-kernel ResNet-50 (NHWC bf16, tony_amd conv/BN/GEMM/residual HIP kernels, the
3-channel 7x7 stem included: ops/csrc/stem.hip), synthetic ImageNet batches generated on the device, SGD-momentum
through ``hvd.DistributedOptimizer``: its bucketed all-reduce (RCCL over xGMI) overlaps the backward
pass and the update is one fused HIP SGD launch per flat buffer.  Reports images/sec over all ranks.

  tony --src_dir tony_amd/jobs --executes hvd_resnet50.py --conf tony.application.framework=horovod \
       --conf tony.worker.instances=8 --conf tony.worker.gpus=1 --conf tony.worker.memory=32g
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import tony_amd.hvd as hvd  # noqa: E402
from tony_amd.jobs.common import Throughput, log, metric, synthetic_images  # noqa: E402
from tony_amd.models.layers import cast_model  # noqa: E402
from tony_amd.models.resnet import resnet50  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=32)
    a = ap.parse_args(argv)
    hvd.init()
    dev = hvd.device()
    on_gpu = dev.type == "cuda"
    dtype = torch.bfloat16 if on_gpu else torch.float32
    if on_gpu:
        torch.backends.cudnn.benchmark = True
    model = cast_model(resnet50(fused=on_gpu), dtype, dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.1 * hvd.size(), momentum=0.9, weight_decay=5e-5)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), bucket_mb=a.bucket_mb)
    x, y = synthetic_images(a.batch_size, a.image_size, 1000, dev, dtype, seed=hvd.rank())
    tp = Throughput(dev)
    for s in range(a.warmup + a.steps):
        if s == a.warmup:
            hvd.barrier()
            tp.start()
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x).float(), y)
        loss.backward()
        opt.step()
        if s >= a.warmup:
            tp.add(a.batch_size)
    rate = float(hvd.allreduce(torch.tensor([tp.rate()]), op=hvd.Sum))
    if hvd.rank() == 0:
        metric(model="resnet50", images_per_sec=rate, size=hvd.size(), batch_per_rank=a.batch_size,
               loss=float(loss))
    log(f"{rate:.1f} images/sec over {hvd.size()} ranks")
    hvd.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
