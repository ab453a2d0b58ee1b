"""Inception-v3 parameter-server training driven by TF_CONFIG -- the headline job
(BASELINE.json: "Inception-v3 TF ParameterServerStrategy 1 ps + 4 workers on 4xMI355X").

PS semantics without TensorFlow (SURVEY.md §7.4 hard part 1): the ps tasks of TF_CONFIG own the
variables and apply the optimizer, workers push gradients and pull variables every step.

``--ps-mode colocated`` (default when the ps tasks have no GPU, not even a shared one:
    ``tony.amd.ps-share-gpu=false``)
    Each worker GPU hosts one shard of the variables: push = RCCL reduce-scatter over xGMI, apply
    = the fused HIP SGD on the shard's fp32 master copy, pull = all-gather.  The ``ps`` tasks of
    the cluster spec do what a TF ps does once the graph is placed -- ``server.join()`` -- and are
    stopped by the coordinator when training ends (ps is untracked by default).
``--ps-mode dedicated`` (default when the ps tasks have a GPU: ``tony.ps.gpus`` >= 1, or TonY's
    default 0-GPU ps placed on a worker's GPU, shared -- ``tony.amd.ps-share-gpu``, exported to every
    task as TONY_PS_SHARED_GPU -- so "1 ps + 4 workers" runs on 4 GPUs)
    The ps task(s) join the group and own the variables.  On GPUs the data plane is the xGMI one of
    parallel/ps_plane.py: workers store gradients straight into the ps GPU's receive windows, the ps
    applies the fused optimizer as they land and stores the new variables straight into every
    worker's landing window.  ``--async`` gives TF's default asynchronous PS (each push applied on
    arrival).

The step (forward, loss, backward, push/apply/pull) runs eagerly with the bucketed push/apply/pull
overlapped with backward, or replayed as a HIP graph (``--graph``).

Checkpoint / resume: with ``--save-steps K`` every rank writes its own PS shard
(fp32 master + momentum of the variables it owns, the variables, its BN running statistics) every K
steps (utils/checkpoint.py, sharded); a relaunched gang (``tony.am.retry-count`` > 0, SESSION_ID > 0)
resumes from the newest step complete on every rank.  ``--fail-at-step S`` is a test hook: in the
first session, worker 1 exits at step S (the TEST_WORKER_TERMINATION idea, mid-training).

  tony --src_dir tony_amd/jobs --executes inception_ps.py --conf tony.ps.instances=1 \
       --conf tony.worker.instances=4 --conf tony.worker.gpus=1 --conf tony.worker.memory=32g
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tony_amd.jobs.common import Throughput, log, metric, synthetic_images, working_dir  # noqa: E402
from tony_amd.parallel import bootstrap  # noqa: E402
from tony_amd.parallel.ps import ParameterServer  # noqa: E402
from tony_amd.parallel.tf_config import TFConfig  # noqa: E402
from tony_amd.parallel.trainer import Trainer  # noqa: E402
from tony_amd.utils.checkpoint import CheckpointManager, resume_step  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ps-mode", default="auto", choices=["auto", "colocated", "dedicated"])
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--image-size", type=int, default=299)
    ap.add_argument("--no-graph", action="store_true", help="(default) issue the step eagerly")
    ap.add_argument("--graph", action="store_true", help="replay the step as a HIP graph")
    ap.add_argument("--checkpoint-dir", default=None, help="default: <job dir>/inception_ps")
    ap.add_argument("--save-steps", type=int, default=0, help="checkpoint every K steps (0: never)")
    ap.add_argument("--fail-at-step", type=int, default=-1, help="test hook (session 0, worker 1)")
    ap.add_argument("--async", dest="async_ps", action="store_true",
                    help="asynchronous PS (dedicated mode): every worker push applied on its own on arrival")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute precision on GPU: bf16 (default) or fp32 -- the reference job's precision "
                         "(mnist_distributed.py: fp32 variables and compute): fp32 activations, variables and "
                         "pushed gradients, each conv / GEMM product as an x3 split over the bf16 MFMA kernels")
    a = ap.parse_args(argv)
    tc = TFConfig.from_env()
    on_gpu = torch.cuda.is_available()
    mode = a.ps_mode
    if mode == "auto":  # every task must decide the same way: only from the shared conf / env
        ps_gpus = int(os.environ.get("TONY_PS_GPUS", "0") or 0)
        # a 0-GPU ps placed on a worker's GPU (tony.amd.ps-share-gpu, the default) owns the variables
        shared = os.environ.get("TONY_PS_SHARED_GPU", "0") == "1"
        mode = os.environ.get("TONY_PS_MODE") or (
            "dedicated" if ps_gpus > 0 or shared or not on_gpu else "colocated")
    if mode == "colocated":
        if tc.task_type == "ps":
            log("colocated PS: variables are sharded over the worker GPUs; ps task joins (waits) until stopped")
            while True:
                time.sleep(3600)
        tc = tc.without_ps()
    rank, world, dev = bootstrap.init_from_tf_config(tc)
    torch.manual_seed(1000 + rank)  # dropout masks: reproducible per rank (and restored on resume)
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.models.layers import cast_model

    x3 = on_gpu and a.dtype == "fp32"  # reference precision on the x3-split kernels (ops/x3.py)
    dtype = torch.bfloat16 if on_gpu and not x3 else torch.float32
    if on_gpu:
        torch.backends.cudnn.benchmark = True
    if x3:
        model = inception_v3(fused=False, seed=0, precision="fp32").to(dev).to(memory_format=torch.channels_last)
    else:
        model = cast_model(inception_v3(fused=on_gpu, seed=0), dtype, dev).to(memory_format=torch.channels_last)
    ps = ParameterServer(model, optimizer="sgd", lr=0.045, momentum=0.9, weight_decay=4e-5, mode=mode,
                         ps_ranks=tc.ps_ranks if mode == "dedicated" else (0,), dtype=dtype, device=dev,
                         wire_dtype=torch.float32 if dtype == torch.float32 else None,
                         sync=not (a.async_ps and mode == "dedicated"))
    if mode == "dedicated" and not ps.sync and ps.plane is None:
        raise SystemExit("--async needs the xGMI PS data plane (GPU ranks)")

    from tony_amd.ops import cross_entropy  # fused HIP softmax-xent on GPU tensors, torch's on CPU

    def loss_fn(out, y):
        logits, aux = out if isinstance(out, tuple) else (out, None)
        loss = cross_entropy(logits, y)
        if aux is not None:
            loss = loss + 0.4 * cross_entropy(aux, y)
        return loss

    total = a.warmup + a.steps
    ckpt = CheckpointManager(a.checkpoint_dir or working_dir("inception_ps"), save_steps=a.save_steps,
                             sharded=True)
    start = 0
    state = ckpt.restore(device=dev if on_gpu else None)
    if state is not None:
        ps.load_state_dict(state["ps"])
        with torch.no_grad():
            missing = []
            for k, b in model.named_buffers():
                if k in state["buffers"]:
                    b.copy_(state["buffers"][k])
                else:  # a checkpoint older than the buffer (e.g. the dropout step counter): keep the init
                    missing.append(k)
            if missing:
                log(f"checkpoint has no buffers {missing}: kept their initial values")
        torch.set_rng_state(state["rng_cpu"])  # dropout masks continue exactly where they were
        if on_gpu and "rng_cuda" in state:
            torch.cuda.set_rng_state(state["rng_cuda"], dev)
        start = resume_step(state)
        log(f"session {os.environ.get('SESSION_ID', '0')}: resumed from step {start}")

    def save(step, force=False):
        st = {"ps": ps.state_dict(), "buffers": dict(model.named_buffers()), "rng_cpu": torch.get_rng_state()}
        if on_gpu:
            st["rng_cuda"] = torch.cuda.get_rng_state(dev)
        ckpt.save(step, st, force=force)

    # Every rank issues the same sequence of collectives on the default group: the per-step PS
    # collectives (RCCL plane: each bucket's reduce / broadcast), ONE barrier at the first timed
    # step, then the rate all-reduce and the closing barrier.  (The ps task used to run only the
    # per-step collectives and one barrier: its sequence did not match the workers'.)
    timed_from = max(start, a.warmup)
    if mode == "dedicated" and ps.is_ps and not ps.is_worker:
        for s in range(start, total):  # the ps task: apply bucket by bucket as the pushes land
            if s == timed_from:
                dist.barrier()
            ps.step()
            if ckpt.should_save(s + 1):
                save(s + 1)
        if a.save_steps:
            save(total, force=True)
            ckpt.wait()
        if on_gpu:
            torch.cuda.synchronize()
        if ps.plane is not None:
            ps.plane.check_error()
        rate = torch.zeros(1, dtype=torch.float64, device=dev if on_gpu else "cpu")
        dist.all_reduce(rate)  # the workers' images/sec sum (the ps adds none)
        dist.barrier()
        if ps.plane is not None:
            ps.plane.close()
        dist.destroy_process_group()
        return 0

    trainer = Trainer(model, ps, loss_fn, use_graph=on_gpu and a.graph)
    x, y = synthetic_images(a.batch_size, a.image_size, 1000, dev, dtype, seed=rank)
    tp = Throughput(dev)
    timed = 0
    loss = torch.zeros(())
    for s in range(start, total):
        if s == a.fail_at_step and os.environ.get("SESSION_ID", "0") == "0" and tc.task_type == "worker" \
                and tc.task_index == 1:
            log(f"test hook: worker 1 fails at step {s}")
            os._exit(17)
        if s == timed_from:
            dist.barrier()
            tp.start()
        loss = trainer.step(x, y)
        if s >= max(start, a.warmup):
            tp.add(a.batch_size)
            timed += 1
        if ckpt.should_save(s + 1):
            save(s + 1)
    if a.save_steps:
        save(total, force=True)
        ckpt.wait()
    rate = torch.tensor([tp.rate() if timed else 0.0], dtype=torch.float64, device=dev if on_gpu else "cpu")
    dist.all_reduce(rate)
    workers = len(ps.worker_ranks)
    if tc.is_chief or rank == 0:
        from tony_amd.parallel import collectives as coll

        # which data plane moved the gradients / variables, and whether its init-time canary against
        # RCCL passed: a run that fell back must not look like one on the hand plane
        metric(model="inception_v3", images_per_sec=float(rate), workers=workers, ps_mode=mode, loss=float(loss),
               dtype="fp32" if dtype == torch.float32 else "bf16", x3=x3, sync=ps.sync,
               start_step=start, steps=total, plane=_plane_name(ps), verified=coll.data_plane_status(),
               collective_fallbacks=coll.fallback_count())
    log(f"{float(rate):.1f} images/sec total over {workers} workers ({mode} PS)")
    dist.barrier()
    # orderly shutdown: drain the device (side streams included) and tear the process group down before
    # interpreter exit -- one run of this job aborted (exit 134) after reporting, during teardown
    if on_gpu:
        torch.cuda.synchronize()
    if ps.plane is not None:
        ps.plane.check_error()
        ps.plane.close()
    dist.destroy_process_group()
    return 0


def _plane_name(ps) -> str:
    """The data plane the PS traffic took: the xGMI PS plane (dedicated), the xGMI collective kernels
    (colocated, TONY_COLLECTIVE=hip) or the process group's backend (rccl / gloo)."""
    from tony_amd.parallel import collectives as coll

    if ps.plane_kind == "xgmi":
        return "xgmi-ps-plane"
    if coll.data_plane_status().get("xgmi_collectives") == "verified":
        return "xgmi-collectives"
    return "rccl" if dist.get_backend() == "nccl" else dist.get_backend()


if __name__ == "__main__":
    sys.exit(main())
