"""Device and process-group backend of a multi-rank GPU test's ranks.

On a node with at least one GPU per rank every rank owns ``cuda:{rank % device_count}`` and the
ranks meet over RCCL (backend ``nccl``): the xGMI kernels then move bytes over real links and the
canaries compare them with RCCL across devices.  On the one-GPU test box every rank shares
``cuda:0`` over gloo (a rehearsal: IPC, the protocols and the kernels, no link).  The choice is in
the test ids (``placement()``), so a run's log says which one ran.  TONY_TEST_BACKEND overrides the
backend (e.g. gloo on distinct devices).
"""
import os

import torch


def n_devices() -> int:
    return torch.cuda.device_count()  # counts devices without initialising HIP


def distinct(world: int) -> bool:
    return n_devices() >= world


def placement(world: int) -> str:
    return f"{world}r-{'distinct-gpus' if distinct(world) else 'shared-gpu0'}"


def bind(rank: int, world: int):
    """Set this rank's device; returns (device, backend)."""
    n = n_devices()
    idx = rank % n if n >= world else 0
    torch.cuda.set_device(idx)
    backend = os.environ.get("TONY_TEST_BACKEND") or ("nccl" if n >= world else "gloo")
    return torch.device("cuda", idx), backend


def init(rank: int, world: int):
    """bind() + init_process_group on MASTER_ADDR / MASTER_PORT from the environment."""
    import torch.distributed as dist

    dev, backend = bind(rank, world)
    dist.init_process_group(backend, rank=rank, world_size=world, device_id=dev if backend == "nccl" else None)
    return dev, backend
